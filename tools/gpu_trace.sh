#!/bin/bash
# same-box A/B of the C2 bench (default vs IC2_FLR_BLOCKED=0), then a rocprofv3 kernel trace of the default for the
# per-step timeline (tools/trace_step.py: kernel time vs span vs idle gaps).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${AB:-default IC2_FLR_BLOCKED=0 default}; do
  if [ $v = default ]; then e=""; else e=$v; fi
  env $e timeout -k 10 300 python bench.py --cpu-baseline-images 0 --no-roofline --out gpurun_out/ab.json > gpurun_out/ab.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --cpu-baseline-images 0 --no-roofline --steps 5 --warmup 3 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_step.py $f 1e9 | tail -40
