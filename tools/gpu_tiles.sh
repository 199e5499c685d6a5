#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SWEEP_ONLY=s36,s52,s84,s148,s148b,s148c timeout -k 10 400 python tools/sweep_igemm.py "" IC2_IGEMM_TILE=6 IC2_IGEMM_TILE=7 > gpurun_out/sweep_tiles.txt 2>&1 || { cat gpurun_out/sweep_tiles.txt; exit 1; }
cat gpurun_out/sweep_tiles.txt
SWEEP_SET=c4 SWEEP_ONLY=T8,T9,T10,T11 timeout -k 10 400 python tools/sweep_igemm.py "" IC2_IGEMM_KORDER=0 IC2_IGEMM_TILE=6 IC2_IGEMM_TILE=7 > gpurun_out/sweep_tiles_c4.txt 2>&1 || { cat gpurun_out/sweep_tiles_c4.txt; exit 1; }
cat gpurun_out/sweep_tiles_c4.txt
