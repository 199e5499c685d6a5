#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SWEEP_ONLY=e1a,e1b,e2a,e2b,e3a,s276a,s276b,s276c timeout -k 10 400 python tools/sweep_igemm.py "" IC2_HG4=0 IC2_HG4=0,IC2_HGEMM=0 > gpurun_out/sweep_sw2.txt 2>&1 || { cat gpurun_out/sweep_sw2.txt; exit 1; }
cat gpurun_out/sweep_sw2.txt
SWEEP_SET=c4 timeout -k 10 400 python tools/sweep_igemm.py "" IC2_HG4=0 IC2_HG4=0,IC2_HGEMM=0 > gpurun_out/sweep_sw2c4.txt 2>&1 || { cat gpurun_out/sweep_sw2c4.txt; exit 1; }
cat gpurun_out/sweep_sw2c4.txt
