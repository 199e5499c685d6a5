#!/bin/bash
# A/B on the GPU box: focused tests (-k expr), then the bench line under each "ENV=VAL" given, then a
# kernel-trace profile of the default build.   usage: bash tools/gpu_ab.sh "<pytest -k expr>" "A=0" "A=1" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_ab.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then echo "pytest failed ($rc): stopping"; exit $rc; fi
shift
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-images 0 > gpurun_out/bench_$kv.json 2> gpurun_out/bench_$kv.err || { echo "bench $kv failed"; tail -20 gpurun_out/bench_$kv.err; exit 1; }
  echo "$kv $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['achieved'])" gpurun_out/bench_$kv.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-baseline-images 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err
echo "rocprof rc=$?"
