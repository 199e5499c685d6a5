#!/bin/bash
# PMC passes over the fused filtered-lrelu of one SG3-T-256 layer (tools/prof_flr.py <layer>)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcflr2
export TMPDIR=/tmp
LAYER=${1:-8}
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
            "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_ACTIVE_INST_EXP"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcflr2/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_flr.py $LAYER 5 > gpurun_out/pmcflr2/p$i.log 2>&1 || { echo "flr pass $i failed"; tail -3 gpurun_out/pmcflr2/p$i.log; }
done
python3 tools/pmc_agg.py 'gpurun_out/pmcflr2/p*' flrelu | tee gpurun_out/pmc_flr_wide_l$LAYER.txt
