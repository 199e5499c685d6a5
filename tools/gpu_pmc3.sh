#!/bin/bash
# Per-shape conv PMC (MFMA utilisation, stalls, HBM traffic, LDS) over every bench conv shape on the current launch plan.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcs3
export TMPDIR=/tmp
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcs3/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_shapes.py 3 > gpurun_out/pmcs3/p$i.log 2>&1 || { echo "shapes pass $i failed"; tail -3 gpurun_out/pmcs3/p$i.log; exit 1; }
done
python3 tools/pmc_shapes_agg.py 'gpurun_out/pmcs3/p*' 3 > gpurun_out/pmc_shapes3.json
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_shapes3.json'))
for k,v in d.items(): print(k, v['kernel'], v['us_profiled_median'], round(v['gflop']/v['us_profiled_median']*1e3) if v['us_profiled_median'] else None, v.get('mfma_util'), v.get('clock_ghz'), v.get('traffic_x'))
"
