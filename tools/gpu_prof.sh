#!/bin/bash
# focused parity tests (-k "$1"), the C2 bench line, and a rocprofv3 kernel-trace --stats of the C2 bench (tag $2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${2:-cur}
if [ -n "$1" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_$TAG.json > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));r=d['roofline'];print('c2', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline-images 0 --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv \;
python3 $GRAFT_REPO_ROOT/tools/kstats.py $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv 30 2>/dev/null | head -30 || head -25 $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv | cut -c1-150
