#!/bin/bash
# blocked conv -> FLR hand-off: parity tests (FLR, conv layouts, C2 end to end), per-layer FLR A/B, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "flrelu or filtered or nhwc16" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/flr_tests.log 2>&1
rc=$?
tail -3 gpurun_out/flr_tests.log
[ $rc -eq 0 ] || { echo "kernel tests failed ($rc): stopping"; grep -E "^E |Error|FAIL" gpurun_out/flr_tests.log | head -30; exit $rc; }
timeout -k 10 600 python tools/bench_kernels.py flr default "$@" 2>&1 | tee gpurun_out/flr_layers.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2_parity.py -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/c2_parity.log 2>&1
rc=$?
grep "\[c2\]" gpurun_out/c2_parity.log; tail -2 gpurun_out/c2_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --cpu-baseline-images 0 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
