# training-path changes: the training GPU tests, then the C5 bench line
set -o pipefail
mkdir -p gpurun_out/c5c
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_ddp.py > gpurun_out/c5c/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c5c/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 > gpurun_out/c5c/c5.json 2> gpurun_out/c5c/c5.err; echo "c5 rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/c5c/c5.json'));print('C5',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'),d['last_step_losses'])"
timeout -k 10 400 bash tools/gpu_evidence.sh c5c trace5 > gpurun_out/c5c/trace5.log 2>&1; echo "trace5 rc=$?"
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/c5c/c5c_c5_kernel_stats.csv')[0]
r = list(csv.DictReader(open(f)))
tot = sum(float(x['TotalDurationNs']) for x in r)
print('kernel ms per step (13 steps)', round(tot / 1e6 / 13, 3))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs'])):
    n = x['Name']
    if any(k in n for k in ('colsum', 'gnb_', 'reduce_kernel', 'scale_bwd', 'fb_ydot', 'where', 'FillFunctor')):
        print('%7.3f ms %5d calls  %s' % (float(x['TotalDurationNs']) / 1e6 / 13, int(x['Calls']) // 13, n[:110]))
PY
