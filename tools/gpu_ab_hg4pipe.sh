#!/bin/bash
# A/B of the pipelined hg4 instances (IC2_HG4_PIPE mask) on the C2 / C4 benches, same box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm4" -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/hg4p_tests.log 2>&1 || { tail -30 gpurun_out/ab/hg4p_tests.log; exit 1; }
tail -2 gpurun_out/ab/hg4p_tests.log
for cfg in c2 c4; do
  for m in 0 7 0 7; do
    IC2_DEV=1 IC2_HG4_PIPE=$m timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/ab/hg4p_${cfg}_$m.json > gpurun_out/ab/hg4p_${cfg}_$m.log 2>&1 || { tail -20 gpurun_out/ab/hg4p_${cfg}_$m.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/hg4p_${cfg}_$m.json')); pk=d['roofline']['per_kernel']; print('$cfg pipe=$m', d['value'], {k: (v['ms_per_step'], v['executed_tflops']) for k, v in pk.items() if k.startswith('hg4')})"
  done
done
