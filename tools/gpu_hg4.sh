#!/bin/bash
# hg4 (4-wave halo GEMM) on the GPU box: its parity tests, the per-shape sweep (off / default / forced), and the
# C2 bench line with it off and on.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo_gemm or conv_igemm or modconv_prep_batched or layer_api or synthesis_fp32_within" > gpurun_out/pytest_hg4.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_hg4.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_hg4.log | head -20; exit $rc; }
SWEEP_ONLY=${SHAPES:-e1a,e1b,e2a,e2b,e3a,s148b,s148c,s276a,s276b,s276c} timeout -k 10 400 python tools/sweep_igemm.py \
  IC2_HG4=0 IC2_HG4=2 > gpurun_out/sweep_hg4.txt 2>&1 || { cat gpurun_out/sweep_hg4.txt; exit 1; }
cat gpurun_out/sweep_hg4.txt
for v in 0 1; do
  IC2_HG4=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_hg4_$v.json > gpurun_out/bench_hg4_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bench_hg4_$v.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_hg4_$v.json'));r=d['roofline'];print('IC2_HG4=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'])"
done
