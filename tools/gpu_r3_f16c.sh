#!/bin/bash
# C4 parity in bf16 + f16 synthesis, the f16 perturbation test, C4 benches, the platform GEMM probe
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_parity.py tests/test_gpu_c2_parity.py -m gpu -q -rP --timeout 350 \
  --timeout-method thread > gpurun_out/r3f/parity3.log 2>&1 \
&& timeout -k 10 120 python -u tools/gemm_peak_probe.py gpurun_out/r3f/gemm_probe.json > gpurun_out/r3f/gemm.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 3 --cpu-baseline-images 0 \
  --out gpurun_out/r3f/c4_bf16.json > gpurun_out/r3f/c4_bf16.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 3 --precision f16 --cpu-baseline-images 0 \
  --out gpurun_out/r3f/c4_f16.json > gpurun_out/r3f/c4_f16.log 2>&1
rc=$?
grep -E "passed|failed|error|\[c2\]|\[c4\]" gpurun_out/r3f/parity3.log | tail -30
cat gpurun_out/r3f/gemm.log
for f in gpurun_out/r3f/c4*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('flr',{}).get('ms_per_step'))"; done
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3f/parity3.log | head -10; tail -5 gpurun_out/r3f/*.log; }
exit $rc
