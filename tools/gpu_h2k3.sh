# A/B: split-weight f16 on the first 3 encoder blocks (knob IC2_SPLIT_F16_BLOCKS=3) vs the default 2
set -o pipefail
O=gpurun_out/r5h2k3
mkdir -p $O
IC2_DEV=1 IC2_SPLIT_F16_BLOCKS=3 timeout -k 10 300 python -u bench.py > $O/c2_k3.json 2> $O/c2_k3.err && echo "bench k3 ok" &&
python3 -c "import json;d=json.load(open('$O/c2_k3.json'));p=d['parity']['indices'];c=d['secondary']['c4'];q=c['parity']['indices'];print('K3 C2',d['value'],d['ms_per_step'],p['mismatches'],p['max_abs_mean_diff'],'| C4',c['value'],c['ms_per_step'],q['mismatches'],q['max_abs_mean_diff'])" &&
timeout -k 10 300 python -u bench.py > $O/c2_k2.json 2> $O/c2_k2.err && echo "bench k2 ok" &&
python3 -c "import json;d=json.load(open('$O/c2_k2.json'));p=d['parity']['indices'];c=d['secondary']['c4'];q=c['parity']['indices'];print('K2 C2',d['value'],d['ms_per_step'],p['mismatches'],p['max_abs_mean_diff'],'| C4',c['value'],c['ms_per_step'],q['mismatches'],q['max_abs_mean_diff'])"
