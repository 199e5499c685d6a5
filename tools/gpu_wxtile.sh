# Winograd tile sweep on the dominant C2 shapes (IC2_WINO_TWP / IC2_WINO_TH forced; plan default first)
set -o pipefail
mkdir -p gpurun_out/wxtile
export IC2_DEV=1
echo "default: $(timeout -k 10 120 python -u tools/bench_wino.py s84 s148 s148b s148c 2>&1 | grep -o '^s[0-9a-z]*\|plan_wino": "[a-z0-9_]*\|"wino": \[[0-9.]*' | tr '\n' ' ')" || exit 1
for t in "16 8" "14 8" "12 8" "15 4" "8 8" "16 4" "10 8" "30 4"; do
  set -- $t
  echo "twp=$1 th=$2: $(IC2_WINO_TWP=$1 IC2_WINO_TH=$2 timeout -k 10 120 python -u tools/bench_wino.py s84 s148 s148b s148c 2>&1 | grep -o '^s[0-9a-z]*\|"wino": \[[0-9.]*' | tr '\n' ' ')" || exit 1
done
