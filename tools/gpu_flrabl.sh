#!/bin/bash
# FLR ablations on the current build (diagnostic builds give WRONG images; only the FLR ms per step is read)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1 4 16 32 0; do
IC2_FLR_ABL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_abl$v.json > gpurun_out/bench_abl$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_abl$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_abl$v.json'));r=d['roofline'];print('abl=$v', d['value'], d['ms_per_step'], r['flr']['ms_per_step'])"
done
