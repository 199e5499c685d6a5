#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "conv_igemm or halo_gemm" > gpurun_out/pytest_rfl.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_rfl.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_rfl.log | head -20; exit $rc; }
timeout -k 10 400 python tools/sweep_igemm.py "" > gpurun_out/sweep_rfl.txt 2>&1 || { cat gpurun_out/sweep_rfl.txt; exit 1; }
cat gpurun_out/sweep_rfl.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_rfl.json > gpurun_out/bench_rfl.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_rfl.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_rfl.json'));r=d['roofline'];print('c2', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
