#!/bin/bash
# hg4 variants: forced-instance parity, then the per-shape sweep over ring depth / o-tile, then C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IC2_HG4_NS=4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_gemm4" > gpurun_out/pytest_hg4b.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_hg4b.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_hg4b.log | head -20; exit $rc; }
SWEEP_ONLY=e1a,e1b,e2a,e2b,s276a,s276b,s276c timeout -k 10 400 python tools/sweep_igemm.py \
  IC2_HG4=0 IC2_HG4=2 IC2_HG4=2,IC2_HG4_NS=4 IC2_HG4=2,IC2_HG4_BO=128 IC2_HG4=2,IC2_HG4_BO=128,IC2_HG4_NS=4 > gpurun_out/sweep_hg4b.txt 2>&1 || { cat gpurun_out/sweep_hg4b.txt; exit 1; }
cat gpurun_out/sweep_hg4b.txt
for v in IC2_HG4_NS=3 IC2_HG4_NS=4; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_$v.json > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bench_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));r=d['roofline'];print('$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'])"
done
