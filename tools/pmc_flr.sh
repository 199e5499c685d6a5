#!/bin/bash
# PMC passes (each its own rocprofv3 run, --kernel-trace only) over tools/prof_flr.py <layer>
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcflr
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
            "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcflr/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_flr.py "$@" > gpurun_out/pmcflr/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcflr/p$i.log; }
done
echo done
