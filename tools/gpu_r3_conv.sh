#!/bin/bash
# conv-plan change: conv kernels, plan, path, C2/C4 parity tests, then the C2 and C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/conv
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/conv
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_plan.py tests/test_gpu_path.py tests/test_gpu_c2_parity.py tests/test_gpu_c4_parity.py > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -2 $o/tests.txt
for c in c2 c4; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --out $o/$c.json > $o/$c.log 2>&1 || { tail -20 $o/$c.log; exit 1; }
python3 -c "import json; d=json.load(open('$o/$c.json')); pk=d['roofline']['per_kernel']; print('$c', d['value'], d['ms_per_step'], '  '.join(f\"{k}:{v['ms_per_step']:.3f}\" for k,v in pk.items() if 'hg4' in k))"
done
