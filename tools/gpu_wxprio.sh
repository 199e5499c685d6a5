# wave-priority A/B of the Winograd kernel (tools/build_abl.sh winoprio 1 2): base / no setprio / prio on R, twice
set -o pipefail
mkdir -p gpurun_out/wxprio
L=$GRAFT_REPO_ROOT/image_compression_2_amd
for rep in 1 2; do
  for v in base 1 2; do
    if [ $v = base ]; then lib=""; else lib=$L/libic2ops_wxprio$v.so; fi
    echo "$v: $(IC2_DEV=1 IC2_DEV_LIB=$lib timeout -k 10 120 python -u tools/bench_wino.py s84 s148 s148b s148c 2>&1 | grep -o '^s[0-9a-z]*\|"wino": \[[0-9.]*' | tr '\n' ' ')" || exit 1
  done
done
for v in 1 2; do
  IC2_DEV=1 IC2_DEV_LIB=$L/libic2ops_wxprio$v.so timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_wino.py 2>&1 | tail -1
done
