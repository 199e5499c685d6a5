#!/bin/bash
# Round-end evidence on the GPU box: every GPU test, the default bench line (with the CPU baseline), a
# kernel-trace profile of the same command, PMC HBM traffic per conv launch, and the C4 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc): stopping"; exit $rc; fi
timeout -k 10 300 bash tools/pmc_traffic.sh r1_pmc_traffic_c2_bf16_b32 || exit 1
cp gpurun_out/pmc_traffic/r1_pmc_traffic_c2_bf16_b32.json profiles/ || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --cpu-baseline-images 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "c4 bench failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-baseline-images 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
echo "rocprof rc=$?"
