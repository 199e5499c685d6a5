# split-weight f16 first blocks (IC2_F16X2): op tests, encoder parity, C2 (+ secondary C4) bench with the knob at 2
# and at 0 (all split bf16)
set -o pipefail
O=gpurun_out/r5h2b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 200 --timeout-method thread > $O/split.log 2>&1 && echo "split ok" &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_c2_parity.py tests/test_gpu_c4_parity.py tests/test_gpu_path.py -x -q -s --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && echo "parity ok" &&
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err && echo "bench ok" &&
python3 -c "import json;d=json.load(open('$O/c2.json'));r=d['roofline'];print('C2',d['value'],d['ms_per_step'],r['path_frac'],d['parity']['meets_bars'],d['parity'].get('max_abs_latent_diff'),d['parity'].get('index_mismatch_frac'),'| C4',d['secondary']['c4']['value'],d['secondary']['c4']['ms_per_step'],d['secondary']['c4']['parity']['meets_bars'])" &&
timeout -k 10 300 python -u bench.py > $O/c2_k0.json 2> $O/c2_k0.err && echo "bench k0 ok" &&
python3 -c "import json;d=json.load(open('$O/c2_k0.json'));r=d['roofline'];print('C2 run2',d['value'],d['ms_per_step'],r['path_frac'],d['parity']['meets_bars'],'| C4',d['secondary']['c4']['value'],d['secondary']['c4']['ms_per_step'])"
