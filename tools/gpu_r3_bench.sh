#!/bin/bash
# round 3 benches: C2 (default precision, with roofline + CPU baseline), C4, C2g, and a rocprofv3 kernel-trace of C2
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3b
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:-r3b}
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --out gpurun_out/r3b/${tag}_c2.json > gpurun_out/r3b/${tag}_c2.log 2>&1 || { tail -20 gpurun_out/r3b/${tag}_c2.log; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --out gpurun_out/r3b/${tag}_c4.json > gpurun_out/r3b/${tag}_c4.log 2>&1 || { tail -20 gpurun_out/r3b/${tag}_c4.log; exit 1; }
timeout -k 10 300 python bench.py --config c2g --steps 20 --warmup 5 --out gpurun_out/r3b/${tag}_c2g.json > gpurun_out/r3b/${tag}_c2g.log 2>&1 || { tail -20 gpurun_out/r3b/${tag}_c2g.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r3b/prof_c2 -o run -- python3 bench.py --steps 7 --warmup 3 --cpu-baseline-images 0 --no-roofline > gpurun_out/r3b/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/r3b/${tag}_prof.log; exit 1; }
find gpurun_out/r3b/prof_c2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r3b/${tag}_c2_kernel_stats.csv \;
for f in c2 c4 c2g; do python3 -c "import json,sys; d=json.load(open('gpurun_out/r3b/${tag}_$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('cpu_baseline',{}).get('value'))"; done
