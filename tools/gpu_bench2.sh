# two default bench runs (C2 + secondary C4) with parity records
set -o pipefail
O=gpurun_out/${1:-r5b2}
mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python -u bench.py > $O/c2_$i.json 2> $O/c2_$i.err || exit 1
python3 -c "import json;d=json.load(open('$O/c2_$i.json'));p=d['parity']['indices'];c=d['secondary']['c4'];q=c['parity']['indices'];print('C2',d['value'],d['ms_per_step'],p['mismatches'],p['max_abs_mean_diff'],'| C4',c['value'],c['ms_per_step'],q['mismatches'],q['max_abs_mean_diff'])" || exit 1
done
