#!/bin/bash
# Conv iteration on the GPU box: conv parity tests, then the conv-shape sweep (default vs the implicit GEMM
# only), then the default bench line.  Stops on a crash / timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "conv" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
rc=$?
tail -15 gpurun_out/conv_tests.log
[ $rc -eq 0 ] || { echo "conv tests failed ($rc): stopping"; exit $rc; }
timeout -k 10 600 python tools/sweep_igemm.py ${SWEEP_VARIANTS:-"" "IC2_HGEMM=0"} 2>&1 | tee gpurun_out/sweep.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --cpu-baseline-images 0 --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
