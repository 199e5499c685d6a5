#!/bin/bash
# strip FLR: ring DMA issued after the vertical-up barrier (default) vs after the horizontal pass (libic2ops_abl0.so,
# built with -DFM3_EARLY=0); FLR kernel tests first
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/early
export PYTHONUNBUFFERED=1
o=gpurun_out/early
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "flrelu or filtered_lrelu" > $o/kernels.log 2>&1 || { tail -30 $o/kernels.log; exit 1; }
tail -1 $o/kernels.log
for r in 1 2; do
  timeout -k 10 120 python tools/ab_flr.py early >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
  IC2_DEV=1 IC2_DEV_LIB=$GRAFT_REPO_ROOT/image_compression_2_amd/libic2ops_abl0.so timeout -k 10 120 python tools/ab_flr.py late >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
done
grep total $o/ab.txt
