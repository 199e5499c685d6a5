#!/bin/bash
# 8-phase split-K: new parity cases, split / path / C2 / C4 parity tests, A/B vs the 128 x 128 split-K tile
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g8sk
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/g8sk
timeout -k 10 800 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_split.py tests/test_gpu_path.py tests/test_gpu_c2_parity.py tests/test_gpu_c4_parity.py -k "g8_splitk or split or synthesis or encoder or c2 or c4 or layer or compress" > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
tail -1 $o/tests.txt
KNOB=IC2_G8_SPLITK VALS="1 0 1 0" CFGS="c2 c4" STEPS=20 PKF=igemm bash tools/gpu_ab_knob.sh
