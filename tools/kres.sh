#!/bin/bash
# usage: tools/kres.sh file.hip  -> per-kernel VGPR / AGPR / scratch / occupancy / LDS (compile-time resource usage)
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep "remark:" | sed -e 's/ \[-Rpass-analysis=kernel-resource-usage\]//' -e 's/.*remark: *//' |
  awk '/^Function Name:/{n=$3} /^VGPRs:/{v=$2} /^AGPRs:/{ag=$2} /^ScratchSize/{s=$NF} /^Occupancy/{o=$NF}
       /^LDS Size/{print n, "vgpr="v, "agpr="ag, "scratch="s, "occ="o, "lds="$NF}' |
  c++filt | sed -e 's/ic2:://g' -e 's/__hip_bfloat16/bf16/g'
