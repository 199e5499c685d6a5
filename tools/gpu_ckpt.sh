#!/bin/bash
# checkpoint on the GPU box: whole GPU test suite, then the C2 / C4 / C2r bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "GPU tests failed ($rc)"; grep -E "^E |FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for c in c2 c4 c2r; do
  timeout -k 10 400 python bench.py --config $c --cpu-baseline-images 0 --out gpurun_out/bench_$c.json > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['flr']['ms_per_step'], r['frac'], r['path_frac'])"
done
