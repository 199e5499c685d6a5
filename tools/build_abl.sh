#!/bin/bash
# diagnostic library builds with IC2_FM3_ABL ablations of the strip FLR (wrong results; timing only), loaded by
# IC2_DEV=1 IC2_DEV_LIB=<path>:  bash tools/build_abl.sh 1 2 4
set -e
cd "$(dirname "$0")/.."
for abl in "$@"; do
  d=image_compression_2_amd/_build_abl$abl; mkdir -p $d
  objs=""
  for f in image_compression_2_amd/csrc/*.hip; do
    o=$d/$(basename $f .hip).o
    if [ "$(basename $f)" != flrelu_mfma.hip ] && [ ! -f $o ] && [ -f image_compression_2_amd/_build/$(basename $f .hip).o ]; then
      cp image_compression_2_amd/_build/$(basename $f .hip).o $o   # only flrelu_mfma.hip differs
    fi
    if [ "$(basename $f)" = flrelu_mfma.hip ] || [ ! -f $o ]; then
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wno-unused-result -DIC2_FM3_ABL=$abl $EXTRA \
        $( [ "$(basename $f)" = flrelu_mfma.hip ] && echo "-mllvm -amdgpu-mfma-vgpr-form" ) \
        $( [ "$(basename $f)" = flrelu_bwd.hip ] && echo "-mllvm -pragma-unroll-threshold=200000" ) -c $f -o $o &
    fi
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o image_compression_2_amd/libic2ops_abl$abl.so $objs
  echo built image_compression_2_amd/libic2ops_abl$abl.so
done
