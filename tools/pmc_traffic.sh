#!/bin/bash
# HBM traffic of the bench's igemm launches from PMC counters: two rocprofv3 passes (FETCH_SIZE uses 3 TCC
# slots, WRITE_SIZE 2, so they cannot share a pass), --kernel-trace only, then tools/pmc_traffic.py
# aggregates them per launch into profiles/<name>.json (read by bench.py for roofline.traffic).
# usage: bash tools/pmc_traffic.sh <out-json-name> [bench args...]
set -o pipefail
name=${1:-pmc_traffic}; shift
cd $GRAFT_REPO_ROOT && rm -rf gpurun_out/pmc_traffic/p1 gpurun_out/pmc_traffic/p2 && mkdir -p gpurun_out/pmc_traffic
export TMPDIR=/tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $ctr -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_traffic/p$i -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline-images 0 --no-roofline --no-parity "$@" \
    > gpurun_out/pmc_traffic/p$i.log 2>&1 || { echo "pass $i ($ctr) failed"; tail -5 gpurun_out/pmc_traffic/p$i.log; exit 1; }
done
python3 tools/pmc_traffic.py 'gpurun_out/pmc_traffic/p*' gpurun_out/pmc_traffic/$name.json "$@"
