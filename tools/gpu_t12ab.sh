# A/B: 64-wide statistics-epilogue halo GEMM tile (12-row t12 default vs 8-row p3) on the split-weight f16 blocks
set -o pipefail
O=gpurun_out/r5t12
mkdir -p $O
for v in 1 0 1 0; do
IC2_DEV=1 IC2_X3_GN_T12=$v timeout -k 10 300 python -u bench.py --config c4 --cpu-baseline-images 0 --no-parity > $O/c4_t12_$v.json 2> $O/c4_t12_$v.err || exit 1
python3 -c "import json;d=json.load(open('$O/c4_t12_$v.json'));print('t12=$v C4',d['value'],d['ms_per_step'])" || exit 1
done
