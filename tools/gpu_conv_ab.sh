#!/bin/bash
# conv change check: conv parity tests, full per-shape sweep (default plan), C2 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "halo or conv_igemm or torgb or modconv_prep_batched or layer_api or synthesis_fp32_within or encoder" > gpurun_out/pytest_conv.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_conv.log | head -20; exit $rc; }
timeout -k 10 400 python tools/sweep_igemm.py "" > gpurun_out/sweep_conv.txt 2>&1 || { cat gpurun_out/sweep_conv.txt; exit 1; }
cat gpurun_out/sweep_conv.txt
for c in c2 c4; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-images 0 --out gpurun_out/bench_$c.json > gpurun_out/bench_$c.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r['conv_ms_per_step'], r['frac'], r['path_frac'], r['flr']['ms_per_step'])"
done
