#!/bin/bash
# C4 (1024^2, batch 8) PMC HBM traffic per igemm launch, then the c4 bench line that reads it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 bash tools/pmc_traffic.sh r1_pmc_traffic_c4_bf16_b8 --config c4 || exit 1
cp gpurun_out/pmc_traffic/r1_pmc_traffic_c4_bf16_b8.json profiles/ || exit 1
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo "bench failed"; tail -20 gpurun_out/bench_c4.err; exit 1; }
cat gpurun_out/bench_c4.json
