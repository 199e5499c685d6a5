#!/bin/bash
# Round-2h evidence: every GPU test, C2 / C4 bench lines, rocprofv3 kernel stats of the C2 bench, PMC traffic per conv
# launch (C2, C4) and per-shape conv PMC (MFMA utilisation).  Stops on a crash / timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --durations=10 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "^\[c2\]|FAILED|ERROR" gpurun_out/pytest_gpu.log | head -30
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest crashed ($rc)"; exit $rc; }
timeout -k 10 400 python bench.py --out gpurun_out/bench_c2.json > gpurun_out/bench_c2.log 2>&1 || { echo "c2 bench failed"; tail -20 gpurun_out/bench_c2.log; exit 1; }
cat gpurun_out/bench_c2.json
timeout -k 10 400 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_c4.json > gpurun_out/bench_c4.log 2>&1 || { echo "c4 bench failed"; tail -20 gpurun_out/bench_c4.log; exit 1; }
cat gpurun_out/bench_c4.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline-images 0 --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err) || { echo "rocprof failed"; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r2h_c2_kernel_stats.csv \;
timeout -k 10 400 bash tools/pmc_traffic.sh r2h_pmc_traffic_c2_bf16_b32 || exit 1
timeout -k 10 400 bash tools/pmc_traffic.sh r2h_pmc_traffic_c4_bf16_b8 --config c4 || exit 1
timeout -k 10 400 bash tools/gpu_pmc3.sh || exit 1
timeout -k 10 600 python3 -u bench.py --config c5 --steps 10 --warmup 3 --cpu-baseline-images 0 --out gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/bench_c5.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_c5.json'));print('c5', d['value'], d['ms_per_step'])"
