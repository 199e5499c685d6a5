#!/bin/bash
# strip FLR on the 36-wide layers A/B, then C2 / C4 benches with the strip kernel
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/strip
export PYTHONUNBUFFERED=1
o=gpurun_out/strip
timeout -k 10 120 python tools/ab_flr.py strip > $o/ab2.txt 2>&1 || { tail -20 $o/ab2.txt; exit 1; }
IC2_DEV=1 IC2_FLR_WIDE_ALL=1 timeout -k 10 120 python tools/ab_flr.py wideall >> $o/ab2.txt 2>&1 || { tail -20 $o/ab2.txt; exit 1; }
grep -E "_36_|total" $o/ab2.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-baseline-images 0 --out $o/c2.json > $o/c2.log 2>&1 || { tail -20 $o/c2.log; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c4.json > $o/c4.log 2>&1 || { tail -20 $o/c4.log; exit 1; }
for f in c2 c4; do python3 -c "import json; d=json.load(open('$o/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], r['flr']['ms_per_step'], r['flr']['frac_of_hbm_floor'])"; done
