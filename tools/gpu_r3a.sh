#!/bin/bash
# round 3a: split-bf16 encoder, launch-plan coverage, grad-mode inference, C2 parity, bench c2 (default precision)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_split.py \
  tests/test_gpu_plan.py "tests/test_gpu_path.py::test_encoder_full_config_matches_reference" \
  "tests/test_gpu_path.py::test_grad_mode_inference" tests/test_gpu_c2_parity.py > gpurun_out/r3a_pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|\[c2\]|\[plan\]|\[split" gpurun_out/r3a_pytest.log | head -80
[ $rc -eq 0 ] || { tail -60 gpurun_out/r3a_pytest.log; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/r3a_c2.json > gpurun_out/r3a_c2.log 2>&1 || { tail -30 gpurun_out/r3a_c2.log; exit 1; }
cat gpurun_out/r3a_c2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --precision bf16-all --out gpurun_out/r3a_c2_allbf16.json > gpurun_out/r3a_c2b.log 2>&1 || { tail -30 gpurun_out/r3a_c2b.log; exit 1; }
cat gpurun_out/r3a_c2_allbf16.json
