#!/bin/bash
# C5 kernels: GroupNorm backward, encoder backward and the FLR backward tests, then the C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c5b
export PYTHONUNBUFFERED=1
o=gpurun_out/c5b
timeout -k 10 500 python -u -m pytest tests/test_gpu_training.py -m gpu -v -rP --timeout 300 --timeout-method thread \
  -k "conv_backward or group_norm_backward or encoder_backward or flrelu_backward_mfma or training_loss or train_step or scale_ or synthesis_network_gradient or synthesis_layer" > $o/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $o/tests.log | head -20; exit 1; }
grep -E "passed|failed" $o/tests.log | tail -2
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c5.json > $o/c5.log 2>&1 || { tail -20 $o/c5.log; exit 1; }
python3 -c "import json; d=json.load(open('$o/c5.json')); print('c5', d['value'], d['ms_per_step'], d.get('last_step_losses'))"
