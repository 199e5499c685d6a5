#!/bin/bash
# the full GPU suite as the driver runs it (-m gpu), with captured prints of passing tests (-rP) for DESIGN.md
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1120 python -u -m pytest tests -m gpu -v -rP --timeout 900 --timeout-method thread \
  --durations=25 > gpurun_out/r3_suite.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r3_suite.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3_suite.log | head -20; tail -40 gpurun_out/r3_suite.log; }
exit $rc
