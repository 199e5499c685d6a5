#!/bin/bash
# FLR A/B on the GPU box: FLR parity tests, per-layer FLR timings for the default build and the variants named
# on the command line (env settings), then the C2 bench line.  Stops on a crash / timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "flrelu or filtered" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/flr_tests.log 2>&1
rc=$?
tail -3 gpurun_out/flr_tests.log
[ $rc -eq 0 ] || { echo "flr tests failed ($rc): stopping"; tail -30 gpurun_out/flr_tests.log; exit $rc; }
timeout -k 10 600 python tools/bench_kernels.py flr default "$@" 2>&1 | tee gpurun_out/flr_layers.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --cpu-baseline-images 0 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
