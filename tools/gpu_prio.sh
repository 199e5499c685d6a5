#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IC2_HG4_PRIO=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_gemm4" > gpurun_out/pytest_prio.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_prio.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_prio.log | head -20; exit $rc; }
SWEEP_ONLY=e1a,e1b,s276a,s276b,s276c timeout -k 10 400 python tools/sweep_igemm.py IC2_HG4_PRIO=0 IC2_HG4_PRIO=1 IC2_HG4_PRIO=2 IC2_HG4_PRIO=0 IC2_HG4_PRIO=1 IC2_HG4_PRIO=2 > gpurun_out/sweep_prio.txt 2>&1 || { cat gpurun_out/sweep_prio.txt; exit 1; }
cat gpurun_out/sweep_prio.txt
