#!/bin/bash
# split-mode conv + GroupNorm statistics epilogue: split / encoder / parity tests, then C2 and C4 benches + C4 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gnf
export TMPDIR=/tmp PYTHONUNBUFFERED=1
o=gpurun_out/gnf
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_path.py tests/test_gpu_c2_parity.py tests/test_gpu_c4_parity.py -k "split or encoder or c2 or c4" > $o/tests.txt 2>&1 || { tail -40 $o/tests.txt; exit 1; }
grep "fused\|passed\|failed" $o/tests.txt | tail -6
for c in c2 c4; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-images 0 --out $o/$c.json > $o/$c.log 2>&1 || { tail -20 $o/$c.log; exit 1; }
python3 -c "import json; d=json.load(open('$o/$c.json')); pk=d['roofline']['per_kernel']; print('$c', d['value'], d['ms_per_step'], '  '.join(f\"{k}:{v['ms_per_step']:.3f}\" for k,v in pk.items() if 'hg4' in k))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $o/prof_c4 -o run -- python3 bench.py --config c4 --steps 7 --warmup 3 --cpu-baseline-images 0 --no-roofline > $o/prof_c4.log 2>&1 || { tail -20 $o/prof_c4.log; exit 1; }
find $o/prof_c4 -name "*kernel_stats.csv" -exec cp {} $o/c4_kernel_stats.csv \;
echo done
