#!/bin/bash
# A/B of the FLR tile walk order (knob IC2_FLR_ORDER 0 / 1 / 2), C2 bench, same box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
for o in 0 1 2 0 1 2; do
  IC2_DEV=1 IC2_FLR_ORDER=$o timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/ab/flro_$o.json > gpurun_out/ab/flro_$o.log 2>&1 || { tail -20 gpurun_out/ab/flro_$o.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/flro_$o.json')); print('order $o', d['value'], d['roofline']['flr']['ms_per_step'])"
done
