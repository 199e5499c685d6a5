#!/bin/bash
# focused GPU check: selected tests (-k expr), then the bench line and a kernel-trace profile
# usage: bash tools/gpu_quick.sh "<pytest -k expression>"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_quick.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc): stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-images 0 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-baseline-images 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
echo "rocprof rc=$?"
