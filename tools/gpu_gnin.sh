#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "gn_input_fusion or halo_gemm or encoder or c2 or group_norm or gn" > gpurun_out/pytest_gnin.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gnin.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gnin.log | head -20; exit $rc; }
for c in c2 c4; do
for v in 0 1; do
IC2_GN_IN_FUSE=$v timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_${c}_g$v.json > gpurun_out/bench_${c}_g$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${c}_g$v.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_${c}_g$v.json'));r=d['roofline'];print('$c gnin=$v', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
done
done
