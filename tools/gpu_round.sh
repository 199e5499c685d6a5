#!/bin/bash
# Round evidence on the GPU box: every GPU test (C2 parity numbers printed), the default C2 bench line, the C4
# bench line, and a rocprofv3 kernel-trace --stats profile of the C2 bench.  Stops on a crash / timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r2}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --durations=15 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^\[c2\]|\[f16-saturation\]|FAILED|ERROR" gpurun_out/pytest_gpu.log | head -30
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest crashed ($rc)"; exit $rc; }
fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 400 python bench.py --out gpurun_out/bench_c2.json > gpurun_out/bench_c2.log 2>&1 || { echo "c2 bench failed"; tail -20 gpurun_out/bench_c2.log; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 400 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_c4.json > gpurun_out/bench_c4.log 2>&1 || { echo "c4 bench failed"; tail -20 gpurun_out/bench_c4.log; exit 1; }
cat gpurun_out/bench_c4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline-images 0 --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
echo "rocprof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv \;
head -12 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv | cut -c1-160
