#!/bin/bash
# generic A/B of one IC2_DEV knob: forced-instance conv parity under the knob (TESTK = pytest -k filter), then
# benches alternating knob values.  env: KNOB, VALS ("0 1 0 1"), CFGS ("c2 c4"), STEPS, TESTK
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/ab
if [ -n "$TESTK" ]; then
  env IC2_DEV=1 $KNOB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "$TESTK" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
  tail -1 $o/tests.txt
fi
for c in ${CFGS:-c2 c4}; do i=0; for v in ${VALS:-0 1 0 1}; do i=$((i+1))
  t=${c}_${v}_$i
  env IC2_DEV=1 $KNOB=$v timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-15} --warmup 5 --cpu-baseline-images 0 --out $o/$t.json > $o/$t.log 2>&1 || { tail -20 $o/$t.log; exit 1; }
  python3 -c "import json; d=json.load(open('$o/$t.json')); pk=d['roofline']['per_kernel']; print('$t', d['value'], d['ms_per_step'], '  '.join(f\"{k}:{v['ms_per_step']:.3f}\" for k,v in pk.items() if '${PKF:-hg4}' in k))"
done; done
