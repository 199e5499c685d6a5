#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "modconv or layer_api or synthesis_fp32 or c2 or synthesis_input" > gpurun_out/pytest_fc.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fc.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_fc.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_fc.json > gpurun_out/bench_fc.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_fc.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_fc.json'));r=d['roofline'];print('c2', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_fc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline-images 0 --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/prof_fc.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_fc -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/fc_kernel_stats.csv \;
grep -E "fc_|gap|gn_|reparam|synth_input|torgb|from_rgb|style|oscale" $GRAFT_REPO_ROOT/gpurun_out/fc_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
