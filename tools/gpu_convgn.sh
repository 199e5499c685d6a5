#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1 0 1; do
IC2_CONV_GN=$v timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_cgn$v.json > gpurun_out/bench_cgn$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_cgn$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_cgn$v.json'));r=d['roofline'];print('c4 conv_gn=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'])"
done
for v in 0 1; do
IC2_CONV_GN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_cgn2_$v.json > gpurun_out/bench_cgn2_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_cgn2_$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_cgn2_$v.json'));r=d['roofline'];print('c2 conv_gn=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'])"
done
