#!/bin/bash
# Round-2 PMC evidence: per-shape conv counters (HBM traffic, MFMA utilisation, stalls) over every bench conv
# shape, the same stall / LDS counters for the fused filtered-lrelu on L11, then the CPU baseline rows.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcs gpurun_out/pmcflr
export TMPDIR=/tmp
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcs/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_shapes.py 3 > gpurun_out/pmcs/p$i.log 2>&1 || { echo "shapes pass $i failed"; tail -3 gpurun_out/pmcs/p$i.log; }
done
python3 tools/pmc_shapes_agg.py 'gpurun_out/pmcs/p*' 3 > gpurun_out/pmc_shapes.json && head -c 3000 gpurun_out/pmc_shapes.json
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
            "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcflr/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_flr.py 11 5 > gpurun_out/pmcflr/p$i.log 2>&1 || { echo "flr pass $i failed"; tail -3 gpurun_out/pmcflr/p$i.log; }
done
python3 tools/pmc_agg.py 'gpurun_out/pmcflr/p*' flrelu | tee gpurun_out/pmc_flr_l11.txt
timeout -k 10 600 python tools/cpu_baseline.py > gpurun_out/cpu_baseline.log 2>&1; tail -2 gpurun_out/cpu_baseline.log
