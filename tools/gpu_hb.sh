#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IC2_HG4_HB=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_gemm4" > gpurun_out/pytest_hb.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_hb.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_hb.log | head -20; exit $rc; }
SWEEP_ONLY=e1a,e1b,s276a,s276b,s276c timeout -k 10 400 python tools/sweep_igemm.py IC2_HG4_HB=0 IC2_HG4_HB=1 IC2_HG4_HB=0 IC2_HG4_HB=1 > gpurun_out/sweep_hb.txt 2>&1 || { cat gpurun_out/sweep_hb.txt; exit 1; }
cat gpurun_out/sweep_hb.txt
SWEEP_SET=c4 SWEEP_ONLY=E1a,E1b,T9,T11 timeout -k 10 400 python tools/sweep_igemm.py IC2_HG4_HB=0 IC2_HG4_HB=1 > gpurun_out/sweep_hb_c4.txt 2>&1 || { cat gpurun_out/sweep_hb_c4.txt; exit 1; }
cat gpurun_out/sweep_hb_c4.txt
