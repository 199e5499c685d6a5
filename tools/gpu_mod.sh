#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "modconv_prep_batched or layer_api or synthesis_fp32_within or c2 or halo_kernel" > gpurun_out/pytest_mod.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_mod.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_mod.log | head -20; exit $rc; }
SWEEP_ONLY=e0a,e0b,e3a,e3b,e4,s36,s52 timeout -k 10 400 python tools/sweep_igemm.py "" IC2_IGEMM_TILE=3 IC2_IGEMM_TILE=1 \
  IC2_HG4=2,IC2_HG4_MAXC=512 > gpurun_out/sweep_small.txt 2>&1 || { cat gpurun_out/sweep_small.txt; exit 1; }
cat gpurun_out/sweep_small.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_mod.json > gpurun_out/bench_mod.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_mod.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_mod.json'));r=d['roofline'];print('c2', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
