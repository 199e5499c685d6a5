#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_gemm4" > gpurun_out/pytest_c4conv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_c4conv.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_c4conv.log | head -20; exit $rc; }
SWEEP_SET=c4 timeout -k 10 500 python tools/sweep_igemm.py "" IC2_HG4_HCONV=1 IC2_HG4=2 > gpurun_out/sweep_c4.txt 2>&1 || { cat gpurun_out/sweep_c4.txt; exit 1; }
cat gpurun_out/sweep_c4.txt
SWEEP_ONLY=e0a,e0b timeout -k 10 300 python tools/sweep_igemm.py "" IC2_HG4_HCONV=1 > gpurun_out/sweep_e0.txt 2>&1 || { cat gpurun_out/sweep_e0.txt; exit 1; }
cat gpurun_out/sweep_e0.txt
