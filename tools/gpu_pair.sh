# hg4 PAIR (tap-major hi / lo steps of the split-weight f16 statistics kernels): op tests, then C4 / C2 A/B against
# the plain-K-order diagnostic build (libic2ops_hg4pair0.so), alternating on one box
set -o pipefail
O=gpurun_out/r5pair
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v -s --timeout 200 --timeout-method thread -k "f16x2 or split_encoder" > $O/split.log 2>&1 || { echo "split tests failed"; grep -E "^E |FAILED" $O/split.log | head; exit 1; }
grep -E "fused" $O/split.log | grep vs | head -4
for v in pair plain pair plain; do
  if [ $v = plain ]; then env="IC2_DEV=1 IC2_DEV_LIB=image_compression_2_amd/libic2ops_hg4pair0.so"; else env=""; fi
  env $env timeout -k 10 300 python -u bench.py --cpu-baseline-images 0 > $O/c2_$v.json 2> $O/c2_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_$v.json'));c=d['secondary']['c4'];print('$v C2',d['value'],d['ms_per_step'],d['parity']['indices']['mismatches'],'| C4',c['value'],c['ms_per_step'],c['parity']['indices']['mismatches'])" || exit 1
done
