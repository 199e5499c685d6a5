#!/bin/bash
# diagnostic library builds with ablations (wrong results; timing only), loaded by IC2_DEV=1 IC2_DEV_LIB=<path>:
#   bash tools/build_abl.sh [flr] 1 2 4     IC2_FM3_ABL of the strip FLR   -> libic2ops_abl<N>.so
#   bash tools/build_abl.sh hg4 1 2 4       IC2_HG4_ABL of the hg4 conv    -> libic2ops_hg4abl<N>.so
#   bash tools/build_abl.sh wino 1 2 4      IC2_WX_ABL of the Winograd conv -> libic2ops_wxabl<N>.so
#   bash tools/build_abl.sh winostamp 1     IC2_WX_STAMP section timestamps -> libic2ops_wxstamp1.so
#   bash tools/build_abl.sh winosched 1 2   IC2_WX_SCHED schedule variants  -> libic2ops_wxsched<N>.so
#   bash tools/build_abl.sh winoprio 1 2    IC2_WX_PRIO wave-priority variants -> libic2ops_wxprio<N>.so
#   bash tools/build_abl.sh hg4pair 0       IC2_HG4_PAIR=0: split-weight f16 hg4 in the plain K order -> libic2ops_hg4pair0.so
#   (EXTRA="-DIC2_WX_SCHED=2" bash tools/build_abl.sh winostamp 1: stamps of a variant)
set -e
cd "$(dirname "$0")/.."
kind=flr
if [ "$1" = flr ] || [ "$1" = hg4 ] || [ "$1" = wino ] || [ "$1" = winostamp ] || [ "$1" = winosched ] || [ "$1" = winoprio ] || [ "$1" = hg4pair ]; then
  kind=$1; shift
fi
if [ $kind = flr ]; then src=flrelu_mfma.hip; def=IC2_FM3_ABL; tag=abl;
elif [ $kind = wino ]; then src=wino.hip; def=IC2_WX_ABL; tag=wxabl;
elif [ $kind = winostamp ]; then src=wino.hip; def=IC2_WX_STAMP; tag=wxstamp;
elif [ $kind = winosched ]; then src=wino.hip; def=IC2_WX_SCHED; tag=wxsched;
elif [ $kind = winoprio ]; then src=wino.hip; def=IC2_WX_PRIO; tag=wxprio;
elif [ $kind = hg4pair ]; then src=igemm.hip; def=IC2_HG4_PAIR; tag=hg4pair;
else src=igemm.hip; def=IC2_HG4_ABL; tag=hg4abl; fi
for abl in "$@"; do
  d=image_compression_2_amd/_build_$tag$abl; mkdir -p $d
  objs=""
  for f in image_compression_2_amd/csrc/*.hip; do
    o=$d/$(basename $f .hip).o
    b=image_compression_2_amd/_build/$(basename $f .hip).o
    if [ "$(basename $f)" != $src ] && [ -f $b ] && { [ ! -f $o ] || [ $b -nt $o ]; }; then
      cp -p $b $o   # only $src differs (refreshed whenever the default build's object is newer)
    fi
    if [ "$(basename $f)" = $src ] || [ ! -f $o ]; then
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wno-unused-result -D$def=$abl $EXTRA \
        $( [ "$(basename $f)" = flrelu_mfma.hip ] && echo "-mllvm -amdgpu-mfma-vgpr-form" ) \
        $( [ "$(basename $f)" = flrelu_bwd.hip ] && echo "-mllvm -pragma-unroll-threshold=200000" ) -c $f -o $o &
    fi
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o image_compression_2_amd/libic2ops_$tag$abl.so $objs
  echo built image_compression_2_amd/libic2ops_$tag$abl.so
done
