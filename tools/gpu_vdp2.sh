#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IC2_FLR_ABL=128 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "flrelu_nhwc_bf16" > gpurun_out/pytest_vdp2.log 2>&1 || { tail -5 gpurun_out/pytest_vdp2.log; exit 1; }
tail -1 gpurun_out/pytest_vdp2.log
for v in 128 0 128 0; do
IC2_FLR_ABL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_vdp2_$v.json > gpurun_out/bench_vdp2_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_vdp2_$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_vdp2_$v.json'));r=d['roofline'];print('abl=$v', d['value'], d['ms_per_step'], r['flr']['ms_per_step'])"
done
