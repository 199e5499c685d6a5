#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "flrelu or c2 or saturation or synthesis_fp32 or nhwc16" > gpurun_out/pytest_vdp.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_vdp.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_vdp.log | head -20; exit $rc; }
grep -E "^\[c2\]" gpurun_out/pytest_vdp.log | head
for c in c2 c4; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_vdp_$c.json > gpurun_out/bench_vdp_$c.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_vdp_$c.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_vdp_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'], r['flr']['frac_of_bound'])"
done
