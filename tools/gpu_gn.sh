#!/bin/bash
# fused conv + GN statistics: kernel tests, encoder parity, C2 / C4 A/B (IC2_CONV_GN=0 vs fused)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_kernels.py $R/tests/test_gpu_path.py -x -q --timeout 200 --timeout-method thread -k "conv3x3_gn or group_norm or encoder" > $R/gpurun_out/gn_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/gn_tests.log; exit 1; }
tail -2 $R/gpurun_out/gn_tests.log
for cfg in c4 c2; do
  for v in 0 1; do
    IC2_CONV_GN=$v timeout -k 10 300 python3 -u $R/bench.py --config $cfg --steps 20 --warmup 5 --cpu-baseline-images 0 --no-roofline > $R/gpurun_out/gn_${cfg}_$v.json 2>$R/gpurun_out/gn_${cfg}_$v.err || { echo "bench failed"; tail -20 $R/gpurun_out/gn_${cfg}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/gn_${cfg}_$v.json')); print('$cfg IC2_CONV_GN=$v', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
