#!/bin/bash
# round-2f checks: PMC traffic per conv launch on the channel-major K order (C2, C4), C5 training bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_traffic.sh r2f_pmc_traffic_c2_bf16_b32 || exit 1
timeout -k 10 400 bash tools/pmc_traffic.sh r2f_pmc_traffic_c4_bf16_b8 --config c4 || exit 1
timeout -k 10 600 python3 -u bench.py --config c5 --steps 10 --warmup 3 --cpu-baseline-images 0 --out gpurun_out/c5.json > gpurun_out/c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c5.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c5.json'));print('c5', d['value'], d['ms_per_step'])"
