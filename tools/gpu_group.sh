#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SWEEP_ONLY=s52,s84,s148,s148b,s148c timeout -k 10 400 python tools/sweep_igemm.py "" IC2_IGEMM_GROUP=2 IC2_IGEMM_GROUP=4 IC2_IGEMM_GROUP=16 > gpurun_out/sweep_group.txt 2>&1 || { cat gpurun_out/sweep_group.txt; exit 1; }
cat gpurun_out/sweep_group.txt
