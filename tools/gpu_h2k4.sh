# A/B: split-weight f16 on the first 4 encoder blocks (knob IC2_SPLIT_F16_BLOCKS=4) vs the default 3, same box
set -o pipefail
O=gpurun_out/r5h2k4
mkdir -p $O
for k in 4 3; do
IC2_DEV=1 IC2_SPLIT_F16_BLOCKS=$k timeout -k 10 300 python -u bench.py > $O/c2_k$k.json 2> $O/c2_k$k.err || exit 1
python3 -c "import json;d=json.load(open('$O/c2_k$k.json'));p=d['parity']['indices'];c=d['secondary']['c4'];q=c['parity']['indices'];print('K$k C2',d['value'],d['ms_per_step'],p['mismatches'],p['max_abs_mean_diff'],'| C4',c['value'],c['ms_per_step'],q['mismatches'],q['max_abs_mean_diff'])" || exit 1
done
