#!/bin/bash
# the f16 synthesis mode: its kernel tests (conv instances, ToRGB, filtered lrelu with f16 output), the launch-plan
# parity over the benched f16 workloads, the C2 parity in f16, then C2 benches bf16 vs f16
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rP --timeout 300 --timeout-method thread \
  -k "float16 or f16 or conv_igemm or torgb or flrelu_nhwc_bf16" > gpurun_out/r3f/kern.log 2>&1 \
&& timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_c2_parity.py -m gpu -x -q -rP --timeout 300 \
  --timeout-method thread > gpurun_out/r3f/parity.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/r3f/c2_bf16.json \
  > gpurun_out/r3f/c2_bf16.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --precision f16 --cpu-baseline-images 0 \
  --out gpurun_out/r3f/c2_f16.json > gpurun_out/r3f/c2_f16.log 2>&1
rc=$?
for f in gpurun_out/r3f/*.log; do echo "== $f"; grep -E "passed|failed|error|\[c2\]" $f | tail -12; done
[ $rc -eq 0 ] || { for f in gpurun_out/r3f/*.log; do grep -E "FAILED|Error" $f | head -10; done; }
exit $rc
