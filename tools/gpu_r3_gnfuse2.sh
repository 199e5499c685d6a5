#!/bin/bash
# fused split conv + GN statistics over image chunks: split tests, C4 parity, C4 A/B fused vs separate
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gnf2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/gnf2
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_c4_parity.py > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
grep "fused\|passed\|failed" $o/tests.txt | tail -6
KNOB=IC2_X3_GN VALS="1 0 1 0" CFGS="c4" STEPS=20 bash tools/gpu_ab_knob.sh
