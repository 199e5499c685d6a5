#!/bin/bash
# fused conv+GN statistics and the fused synthesis-layer backward: tests, A/B benches, C5 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_training.py -x -q -s --timeout 300 --timeout-method thread -k "scale_backward or flrelu_backward_kernel or synthesis_layer_gradients or synthesis_network_gradient or compressor_training or train_step" > $R/gpurun_out/r2b_train.log 2>&1 || { echo "train tests failed"; grep -E "^E |Error|rel grad|passed|failed" $R/gpurun_out/r2b_train.log | head -30; exit 1; }
grep -E "rel grad|passed|failed" $R/gpurun_out/r2b_train.log | cut -c1-200
bash $R/tools/gpu_gn.sh || exit 1
STEPS=10 CPUB=0 bash $R/tools/gpu_c5.sh
