#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_kernel or gn_input or conv_gn or encoder_full or 1024" > gpurun_out/pytest_hcv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_hcv.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_hcv.log | head -20; exit $rc; }
SWEEP_ONLY=e_rgb,e0a,e0b timeout -k 10 300 python tools/sweep_igemm.py "" > gpurun_out/sweep_hcv.txt 2>&1 || { cat gpurun_out/sweep_hcv.txt; exit 1; }
SWEEP_SET=c4 SWEEP_ONLY=E_rgb,E0a,E0b,T11,T12,T13 timeout -k 10 300 python tools/sweep_igemm.py "" >> gpurun_out/sweep_hcv.txt 2>&1 || { cat gpurun_out/sweep_hcv.txt; exit 1; }
cat gpurun_out/sweep_hcv.txt
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_hcv_c4.json > gpurun_out/bench_hcv.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_hcv.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_hcv_c4.json'));r=d['roofline'];print('c4', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
