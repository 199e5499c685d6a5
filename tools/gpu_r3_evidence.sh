#!/bin/bash
# round-3 bench evidence: C2 in every precision, C4, C2g, C5, and rocprofv3 kernel traces of C2 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:-r3e}
o=gpurun_out/$1
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --out $o/${tag}_$n.json > $o/${tag}_$n.log 2>&1 || { tail -20 $o/${tag}_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('$o/${tag}_$n.json')); r=d.get('roofline',{}); print('$n', d['value'], d['ms_per_step'], r.get('frac'), r.get('flr',{}).get('ms_per_step'), d.get('cpu_baseline',{}).get('value'))"
}
run c2 --steps 50 --warmup 10
run c2_bf16all --precision bf16-all --steps 50 --warmup 10 --cpu-baseline-images 0
run c2_f16 --precision f16 --steps 50 --warmup 10 --cpu-baseline-images 0
run c4 --config c4 --steps 20 --warmup 5
run c2g --config c2g --steps 20 --warmup 5
run c5 --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0
for cfg in c2 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $o/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 7 --warmup 3 --cpu-baseline-images 0 --no-roofline > $o/${tag}_prof_$cfg.log 2>&1 || { tail -20 $o/${tag}_prof_$cfg.log; exit 1; }
  find $o/prof_$cfg -name "*kernel_stats.csv" -exec cp {} $o/${tag}_${cfg}_kernel_stats.csv \;
done
echo done
