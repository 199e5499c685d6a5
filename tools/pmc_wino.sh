#!/bin/bash
# PMC passes (each its own rocprofv3 run, --kernel-trace only) over tools/prof_conv.py with PC_WINO=1: the direct
# f16 implicit GEMM and the Winograd kernel on the same conv; aggregate with
#   python tools/pmc_agg.py 'gpurun_out/pmcw/p*' wino_fx   /   ... igemm8_og2_f16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcw
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES TA_BUSY_avr TA_TA_BUSY_sum" "FETCH_SIZE"; do
  i=$((i+1))
  PC_DT=f16 PC_WINO=1 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcw/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_conv.py "$@" > gpurun_out/pmcw/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcw/p$i.log; exit 1; }
done
for k in wino_fx igemm8_og2_f16; do echo "== $k"; python3 tools/pmc_agg.py 'gpurun_out/pmcw/p*' $k; done
