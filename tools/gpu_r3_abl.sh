#!/bin/bash
# strip FLR ablations (diagnostic libraries from tools/build_abl.sh; wrong results, timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl
export PYTHONUNBUFFERED=1
o=gpurun_out/abl
timeout -k 10 120 python tools/ab_flr.py default > $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
for a in ${ABLS:-1 2 4}; do
  IC2_DEV=1 IC2_DEV_LIB=$GRAFT_REPO_ROOT/image_compression_2_amd/libic2ops_abl$a.so timeout -k 10 120 python tools/ab_flr.py abl$a >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
done
timeout -k 10 120 python tools/ab_flr.py default >> $o/ab.txt 2>&1 || { tail -20 $o/ab.txt; exit 1; }
grep total $o/ab.txt
