# final-tree records: full GPU pytest, smoke(), C2 (+secondary C4), C4, C5 bench lines
set -o pipefail
O=gpurun_out/${1:-r5f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err || { echo "c2 failed"; tail -20 $O/c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c2.json'));r=d['roofline'];print('C2',d['value'],d['ms_per_step'],r['frac'],r['path_frac'],r.get('traffic'),r.get('traffic_stale'),d['parity']['meets_bars'],'| C4',d['secondary']['c4']['value'],d['secondary']['c4']['ms_per_step'],d['secondary']['c4']['parity']['meets_bars'],'| cpu',d['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --config c4 > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail -20 $O/c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c4.json'));r=d['roofline'];print('C4',d['value'],d['ms_per_step'],r['frac'],r.get('path_frac'),r.get('traffic'),r.get('traffic_stale'))"
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));print('C5',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d['last_step_losses'])"
