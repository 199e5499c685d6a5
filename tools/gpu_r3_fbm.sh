#!/bin/bash
# MFMA filtered-lrelu backward: kernel + training-path tests, then the C5 bench A/B against the f32 kernel
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fbm
export PYTHONUNBUFFERED=1
o=gpurun_out/fbm
timeout -k 10 500 python -u -m pytest tests/test_gpu_training.py -m gpu -v -rP --timeout 300 --timeout-method thread \
  -k "flrelu_backward_mfma or flrelu_backward_kernel or synthesis_network_gradient or training_loss or train_step" > $o/tests.log 2>&1 || { grep -E "rel err|PASS|FAIL|Error" $o/tests.log | tail -30; tail -30 $o/tests.log; exit 1; }
grep -E "rel err|passed|failed" $o/tests.log | tail -40
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c5.json > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
IC2_DEV=1 IC2_FLRB_MFMA=0 timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c5_f32.json > $o/c5_f32.log 2>&1 || { tail -20 $o/c5_f32.log; exit 1; }
for f in c5 c5_f32; do python3 -c "import json; d=json.load(open('$o/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('last_step_losses'))"; done
