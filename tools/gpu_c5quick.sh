# the shared-trunk training step: its equivalence tests, the training tests, then the C5 bench line
set -o pipefail
mkdir -p gpurun_out/c5q
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_ddp.py > gpurun_out/c5q/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -o "shared trunk.*" gpurun_out/c5q/pytest.log | head -3; tail -3 gpurun_out/c5q/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 > gpurun_out/c5q/c5.json 2> gpurun_out/c5q/c5.err; echo "c5 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/c5q/c5.json'));print('C5',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d['last_step_losses'])"
