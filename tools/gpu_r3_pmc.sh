#!/bin/bash
# round 3 PMC: HBM traffic (two passes) for C2 and C4 in the default precision; $1 = file tag (default r3)
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "c2:32" "c4:8"; do
  c=${cfg%%:*}; b=${cfg##*:}
  rm -rf gpurun_out/pmc_traffic
  bash tools/pmc_traffic.sh ${1:-r3}_pmc_traffic_${c}_bf16_b${b} --config $c || exit 1
  mkdir -p gpurun_out/r3pmc && cp gpurun_out/pmc_traffic/${1:-r3}_pmc_traffic_${c}_bf16_b${b}.json gpurun_out/r3pmc/
done
