#!/bin/bash
# f16 synthesis after the compensated f16 tap rounding: FLR kernel tests, C2 parity (bf16 + f16), C2 benches
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rP --timeout 200 --timeout-method thread \
  -k "flrelu or f16_saturation" > gpurun_out/r3f/kern2.log 2>&1 \
&& timeout -k 10 300 python -u -m pytest tests/test_gpu_c2_parity.py -m gpu -q -rP --timeout 250 \
  --timeout-method thread > gpurun_out/r3f/parity2.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/r3f/c2_bf16.json \
  > gpurun_out/r3f/c2_bf16.log 2>&1 \
&& timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --precision f16 --cpu-baseline-images 0 \
  --out gpurun_out/r3f/c2_f16.json > gpurun_out/r3f/c2_f16.log 2>&1
rc=$?
for f in gpurun_out/r3f/kern2.log gpurun_out/r3f/parity2.log; do echo "== $f"; grep -E "passed|failed|error|\[c2\]" $f | tail -14; done
for f in gpurun_out/r3f/*.json; do echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['roofline']['frac'], d['roofline'].get('flr',{}).get('ms_per_step'))"; done
[ $rc -eq 0 ] || { for f in gpurun_out/r3f/*2.log; do grep -E "FAILED|Error" $f | head -10; done; }
exit $rc
