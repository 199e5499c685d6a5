#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_traffic
timeout -k 10 400 bash tools/pmc_traffic.sh r2h_pmc_traffic_c2_bf16_b32 || exit 1
