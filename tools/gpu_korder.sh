#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IC2_IGEMM_KORDER=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "conv_igemm" > gpurun_out/pytest_korder.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_korder.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_korder.log | head -20; exit $rc; }
SWEEP_ONLY=e3a,e3b,s36,s52,s84,s148,s148b,s148c timeout -k 10 400 python tools/sweep_igemm.py IC2_IGEMM_KORDER=0 IC2_IGEMM_KORDER=1 > gpurun_out/sweep_korder.txt 2>&1 || { cat gpurun_out/sweep_korder.txt; exit 1; }
cat gpurun_out/sweep_korder.txt
for v in 0 1; do
IC2_IGEMM_KORDER=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_k$v.json > gpurun_out/bench_k$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_k$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_k$v.json'));r=d['roofline'];print('korder=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
done
