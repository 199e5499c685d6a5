#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "split_384 or conv_igemm" > gpurun_out/pytest_split.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_split.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_split.log | head -20; exit $rc; }
SWEEP_ONLY=s148,s148b timeout -k 10 300 python tools/sweep_igemm.py IC2_IGEMM_SPLIT=0 "" IC2_IGEMM_SPLIT=0 "" > gpurun_out/sweep_split.txt 2>&1 || { cat gpurun_out/sweep_split.txt; exit 1; }
SWEEP_SET=c4 SWEEP_ONLY=T8 timeout -k 10 300 python tools/sweep_igemm.py IC2_IGEMM_SPLIT=0 "" >> gpurun_out/sweep_split.txt 2>&1 || { cat gpurun_out/sweep_split.txt; exit 1; }
cat gpurun_out/sweep_split.txt
for v in 0 1; do
IC2_IGEMM_SPLIT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_split$v.json > gpurun_out/bench_split$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_split$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_split$v.json'));r=d['roofline'];print('split=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
done
