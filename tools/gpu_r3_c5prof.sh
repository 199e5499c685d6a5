#!/bin/bash
# C5 bench + rocprofv3 kernel trace of the training step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c5p2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/c5p2
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c5.json > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $o/prof -o run -- python3 bench.py --config c5 --steps 6 --warmup 2 --cpu-baseline-images 0 --no-roofline > $o/log 2>&1 || { tail -20 $o/log; exit 1; }
find $o/prof -name "*kernel_stats.csv" -exec cp {} $o/c5_kernel_stats.csv \;
python3 -c "import json; d=json.load(open('$o/c5.json')); print(d['value'], d['ms_per_step'], d.get('last_step_losses'))"
