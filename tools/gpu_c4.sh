#!/bin/bash
# C4 (1024^2, batch 8) on the GPU box: the 1024 parity tests, the c4 bench line, a kernel-trace profile of it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "1024 or halo" > gpurun_out/pytest_c4.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_c4.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc): stopping"; exit $rc; fi
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench failed"; tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python $GRAFT_REPO_ROOT/bench.py --config c4 --steps 2 --warmup 1 --cpu-baseline-images 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_c4.err
echo "rocprof rc=$?"
