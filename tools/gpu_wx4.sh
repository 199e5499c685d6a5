# wx4 (one wave per SIMD) Winograd kernel: parity tests with IC2_WINO_K=7, then the microbenchmark v4 vs wx4
set -o pipefail
mkdir -p gpurun_out/wx4
export IC2_DEV=1
IC2_WINO_K=7 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wino.py > gpurun_out/wx4/test.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/wx4/test.log
[ $rc -le 1 ] || exit $rc
IC2_WINO_K=7 timeout -k 10 240 python -u tools/bench_wino.py s52 s84 s148 s148b s148c > gpurun_out/wx4/bench7.log 2>&1 || exit $?
IC2_WINO_K=4 timeout -k 10 240 python -u tools/bench_wino.py s52 s84 s148 s148b s148c > gpurun_out/wx4/bench4.log 2>&1 || exit $?
grep -h '^s' gpurun_out/wx4/bench7.log gpurun_out/wx4/bench4.log | cut -c1-200
