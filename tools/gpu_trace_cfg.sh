#!/bin/bash
# kernel-trace timeline of one bench step of a config: python tools/trace_step.py over rocprofv3's CSV
# usage: bash tools/gpu_trace_cfg.sh <config> [min_us]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-c2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o run -- python3 bench.py --config $CFG --cpu-baseline-images 0 --no-roofline --steps 3 --warmup 2 > gpurun_out/prof_$CFG.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_$CFG.log; exit 1; }
tail -1 gpurun_out/prof_$CFG.log | cut -c1-200
f=$(find gpurun_out/prof_$CFG -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py $f ${2:-100} | tee gpurun_out/trace_$CFG.txt | cut -c1-150
