#!/bin/bash
# PMC passes (each its own rocprofv3 run, --kernel-trace only) over tools/prof_conv.py
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
            "TA_BUSY_avr TA_TA_BUSY_sum" "SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  IC2_DEV=1 IC2_IGEMM_TILE=${TILE:-0} timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_conv.py "$@" > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
echo done
