set -o pipefail
mkdir -p gpurun_out/c5w
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_training.py > gpurun_out/c5w/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c5w/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/c5w/c5.json 2> gpurun_out/c5w/c5.err; echo "c5 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/c5w/c5.json'));print('C5',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d['last_step_losses'])"
