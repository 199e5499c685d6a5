#!/bin/bash
# Round-2 GPU check: the C2 bf16 parity test (numbers printed), every GPU test, the default bench line.
# A test assertion (pytest rc 1) does not stop the script; a crash / timeout / fault does.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2_parity.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/c2_parity.log 2>&1
rc=$?
grep "\[c2\]" gpurun_out/c2_parity.log
tail -3 gpurun_out/c2_parity.log
ok $rc || { echo "c2 parity crashed ($rc): stopping"; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_gpu_c2_parity.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
tail -3 gpurun_out/pytest_gpu.log
ok $rc || { echo "pytest crashed ($rc): stopping"; exit $rc; }
timeout -k 10 400 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
