#!/bin/bash
# strip-streaming filtered lrelu: kernel parity tests, then per-layer A/B against the round-2 tile kernel
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/strip
export PYTHONUNBUFFERED=1
o=gpurun_out/strip
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "flrelu or filtered_lrelu" > $o/kernels.log 2>&1 || { tail -30 $o/kernels.log; exit 1; }
tail -2 $o/kernels.log
timeout -k 10 120 python tools/ab_flr.py strip > $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
IC2_DEV=1 IC2_FLR_STRIP=0 timeout -k 10 120 python tools/ab_flr.py tile >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
timeout -k 10 120 python tools/ab_flr.py strip >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
grep total $o/ab.txt
