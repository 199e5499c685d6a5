#!/bin/bash
# GAP finalize change: encoder parity tests + C4 parity + C4 bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gap
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/gap
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_path.py tests/test_gpu_c4_parity.py -k "encoder or gap or global_avg or c4 or split" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/c4.json > $o/c4.log 2>&1 || { tail -20 $o/c4.log; exit 1; }
python3 -c "import json; d=json.load(open('$o/c4.json')); print('c4', d['value'], d['ms_per_step'])"
