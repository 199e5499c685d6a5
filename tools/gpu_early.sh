#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "flrelu or c2 or saturation or synthesis_fp32 or nhwc16 or 1024_bf16" > gpurun_out/pytest_early.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_early.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_early.log | head -20; exit $rc; }
for v in 0 1 0 1; do
IC2_FLR_EARLY=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_early$v.json > gpurun_out/bench_early$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_early$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_early$v.json'));r=d['roofline'];print('early=$v', d['value'], d['ms_per_step'], r['flr']['ms_per_step'])"
done
