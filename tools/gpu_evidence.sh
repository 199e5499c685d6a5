#!/bin/bash
# Bench evidence for a round: C2 (default precision) and C4/C5 bench lines, rocprofv3 kernel traces (+ --stats) of C2
# and C4 split into timed steps by tools/trace_steps.py, and the PMC HBM traffic of the C2 conv family
# (tools/pmc_traffic.sh).  Each GPU step has its own time limit; the script stops at the first failure.
#   bash tools/gpu_evidence.sh <tag> [tests [K] smoke c2 c4 c5 trace trace5 pmc pmc4]   (default: c2 c4 c5 trace pmc)
# tests: the GPU pytest suite (optionally only `-k K`, K = comma-separated alternatives), smoke: __graft_entry__.smoke(), pmc4: the C4 PMC traffic,
# abwino <tag>: the Winograd conv of image_compression_2_amd/libic2ops_<tag>.so (tools/build_abl.sh) against the default
# library -- tests/test_gpu_wino.py on the variant, then tools/bench_wino.py on both, alternating, two rounds;
# ab <tag> <tests> <shapes>: the same for any variant library, <tests> = comma-separated test files under tests/,
# <shapes> = comma-separated tools/bench_wino.py shapes (its "direct" column times the implicit-GEMM plan).
# (Replaces the round-5 one-shot gpu_*.sh scripts.)
set -o pipefail
cd $GRAFT_REPO_ROOT || exit 1
tag=${1:-r4}; shift
parts=${*:-"c2 c4 c5 trace pmc"}
o=gpurun_out/$tag
mkdir -p $o
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --out $o/${tag}_$n.json > $o/${tag}_$n.log 2>&1 || { tail -20 $o/${tag}_$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('$o/${tag}_$n.json')); r=d.get('roofline',{}); print('$n', d['value'], d['ms_per_step'], r.get('frac'), r.get('path_frac'), r.get('flr',{}).get('ms_per_step'), d.get('cpu_baseline',{}).get('value'))"
}
set -- $parts
while [ $# -gt 0 ]; do
  p=$1; shift
  case $p in
    tests)
      k=""
      # K: a pytest -k expression without spaces, alternatives separated by commas (ddp,wino -> "ddp or wino")
      if [ $# -gt 0 ] && ! [[ " ab abwino smoke c2 c4 c5 trace trace5 pmc pmc4 " == *" $1 "* ]]; then k=${1//,/ or }; shift; fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread ${k:+-k "$k"} \
        > $o/${tag}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $o/${tag}_pytest.log | tail -30; tail -30 $o/${tag}_pytest.log; exit 1; }
      tail -2 $o/${tag}_pytest.log ;;
    abwino)
      v=$1; shift
      IC2_DEV=1 IC2_DEV_LIB=image_compression_2_amd/libic2ops_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py \
        -x -q --timeout 120 --timeout-method thread > $o/${tag}_ab_$v.log 2>&1 || { echo "variant tests failed"; tail -30 $o/${tag}_ab_$v.log; exit 1; }
      tail -1 $o/${tag}_ab_$v.log
      for rnd in 1 2; do
        for lib in libic2ops libic2ops_$v; do
          IC2_DEV=1 IC2_DEV_LIB=image_compression_2_amd/$lib.so timeout -k 10 300 python -u tools/bench_wino.py s52 s84 s148 s148b s148c \
            > $o/${tag}_ab_${lib}_$rnd.log 2>&1 || { echo "bench_wino failed ($lib)"; tail -20 $o/${tag}_ab_${lib}_$rnd.log; exit 1; }
          echo "== $lib round $rnd"; grep -E "wino" $o/${tag}_ab_${lib}_$rnd.log | tail -6
        done
      done ;;
    ab)
      v=$1; tf=$2; shp=$3; shift 3
      files=""; for f in ${tf//,/ }; do files="$files tests/$f"; done
      IC2_DEV=1 IC2_DEV_LIB=image_compression_2_amd/libic2ops_$v.so timeout -k 10 600 python -u -m pytest $files \
        -x -q --timeout 200 --timeout-method thread > $o/${tag}_ab_$v.log 2>&1 || { echo "variant tests failed"; tail -30 $o/${tag}_ab_$v.log; exit 1; }
      tail -1 $o/${tag}_ab_$v.log
      for rnd in 1 2; do
        for lib in libic2ops libic2ops_$v; do
          IC2_DEV=1 IC2_DEV_LIB=image_compression_2_amd/$lib.so timeout -k 10 300 python -u tools/bench_wino.py ${shp//,/ } \
            > $o/${tag}_ab_${lib}_$rnd.log 2>&1 || { echo "bench_wino failed ($lib)"; tail -20 $o/${tag}_ab_${lib}_$rnd.log; exit 1; }
          echo "== $lib round $rnd"; cat $o/${tag}_ab_${lib}_$rnd.log | python3 -c "import sys,json
for l in sys.stdin:
    n,_,j=l.partition(' ')
    if j.startswith('{'): d=json.loads(j); print(n, 'direct', d['direct'], 'wino', d['wino'])"
        done
      done ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/${tag}_smoke.log 2>&1 \
        || { echo "smoke failed"; tail -20 $o/${tag}_smoke.log; exit 1; }
      tail -1 $o/${tag}_smoke.log ;;
    c2) run c2 --steps 50 --warmup 10 ;;
    c4) run c4 --config c4 --steps 20 --warmup 5 ;;
    c5) run c5 --config c5 --steps 20 --warmup 5 --cpu-baseline-images 0 ;;
    trace)
      for cfg in c2 c4; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $o/prof_$cfg -o run -- python3 bench.py --config $cfg --no-secondary \
          --steps 20 --warmup 3 --cpu-baseline-images 0 --no-roofline --no-parity > $o/${tag}_prof_$cfg.log 2>&1 \
          || { tail -20 $o/${tag}_prof_$cfg.log; exit 1; }
        tr=$(find $o/prof_$cfg -name "*kernel_trace.csv" | head -1)
        find $o/prof_$cfg -name "*kernel_stats.csv" -exec cp {} $o/${tag}_${cfg}_kernel_stats.csv \;
        python3 tools/trace_steps.py $tr --warmup 3 --out $o/${tag}_${cfg}_trace_steps.txt > /dev/null || exit 1
        gzip -c $tr > $o/${tag}_${cfg}_kernel_trace.csv.gz
        tail -4 $o/${tag}_${cfg}_trace_steps.txt
      done ;;
    trace5)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $o/prof_c5 -o run -- python3 bench.py --config c5 \
        --steps 10 --warmup 3 --cpu-baseline-images 0 --no-roofline > $o/${tag}_prof_c5.log 2>&1 \
        || { tail -20 $o/${tag}_prof_c5.log; exit 1; }
      find $o/prof_c5 -name "*kernel_stats.csv" -exec cp {} $o/${tag}_c5_kernel_stats.csv \;
      head -25 $o/${tag}_c5_kernel_stats.csv | cut -c1-160 ;;
    pmc) bash tools/pmc_traffic.sh ${tag}_pmc_traffic_c2_f16_b32 --no-secondary || exit 1 ;;
    pmc4) bash tools/pmc_traffic.sh ${tag}_pmc_traffic_c4_f16_b8 --config c4 || exit 1 ;;
  esac
done
echo "[evidence] done"
