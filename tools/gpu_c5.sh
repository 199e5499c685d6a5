#!/bin/bash
# C5 (encoder training step) bench line + rocprof kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
if [ "${PROF_ONLY:-0}" != 1 ]; then
timeout -k 10 600 python3 -u $R/bench.py --config c5 --steps ${STEPS:-10} --warmup 3 --cpu-baseline-images ${CPUB:-1} \
  --out $R/gpurun_out/c5.json > $R/gpurun_out/c5.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $R/gpurun_out/c5.log; exit 1; }
tail -1 $R/gpurun_out/c5.log
fi
rm -rf /tmp/prof_c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d /tmp/prof_c5 -o c5 -- python3 $R/bench.py --config c5 \
  --steps 4 --warmup 2 --cpu-baseline-images 0 --no-roofline > $R/gpurun_out/c5_prof.log 2>&1 || { echo "prof failed rc=$?"; tail -20 $R/gpurun_out/c5_prof.log; exit 1; }
find /tmp/prof_c5 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/c5_kernel_stats.csv \;
head -30 $R/gpurun_out/c5_kernel_stats.csv | cut -d, -f1-8 | cut -c1-200
