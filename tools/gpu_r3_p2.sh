#!/bin/bash
# hg4 taps-per-barrier A/B: forced-instance parity with the P kernels (IC2_HG4_P2 = 1: two taps; 2: two taps +
# 6-slab o64 ring; 3: three taps + 6-slab o64 ring), then C2 / C4 benches default vs each
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p2
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/p2
for v in ${PV:-2 3}; do
IC2_HG4_P2=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "halo_gemm4" > $o/tests$v.txt 2>&1 || { tail -30 $o/tests$v.txt; exit 1; }
tail -1 $o/tests$v.txt
done
b() { # tag p2 config steps
  IC2_DEV=1 IC2_HG4_P2=$2 timeout -k 10 300 python bench.py --config $3 --steps $4 --warmup 5 --cpu-baseline-images 0 --out $o/$1.json > $o/$1.log 2>&1 || { tail -20 $o/$1.log; exit 1; }
  python3 -c "import json; d=json.load(open('$o/$1.json')); pk=d['roofline']['per_kernel']; print('$1', d['value'], d['ms_per_step'], '  '.join(f\"{k}:{v['ms_per_step']:.3f}\" for k,v in pk.items() if 'hg4' in k))"
}
for c in ${CF:-c4 c2}; do for v in 0 1 2 3 1 0; do b ${c}_$v $v $c 15 || exit 1; done; done
