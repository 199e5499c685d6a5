set -o pipefail
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5s/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/r5s/pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/r5s/c2.json 2> gpurun_out/r5s/c2.err; echo "c2 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/r5s/c2.json'));r=d['roofline'];print('C2',d['value'],d['ms_per_step'],r['path_frac'],d['parity']['meets_bars'],'| C4',d['secondary']['c4']['value'],d['secondary']['c4']['ms_per_step'],d['secondary']['c4']['parity']['meets_bars'],'| flr',r['flr']['ms_per_step'],'| cpu',d['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/r5s/c5.json 2> gpurun_out/r5s/c5.err; echo "c5 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/r5s/c5.json'));print('C5',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d['last_step_losses'],d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/r5s/c4.json 2> gpurun_out/r5s/c4.err; echo "c4 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/r5s/c4.json'));r=d['roofline'];print('C4',d['value'],d['ms_per_step'],r.get('traffic'),r.get('traffic_src'),r.get('traffic_stale'))"
