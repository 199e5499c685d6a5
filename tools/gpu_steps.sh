#!/bin/bash
# Runs GPU steps in order, each under its own time limit; stops at the first step that ends in anything but a pass or
# an ordinary test failure (rc 0 / 1): a fault (also one reported as a Python exception), an abort, a crash or a
# time limit ends the call there.
#   bash tools/gpu_steps.sh <outdir> "<seconds> <command>" ...
out=$1; shift
mkdir -p "$out"
i=0
for step in "$@"; do
  i=$((i + 1))
  secs=${step%% *}; cmd=${step#* }
  echo "[gpu_steps] step $i (${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "[gpu_steps] step $i rc=$rc"; tail -3 "$out/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_steps] stopping after rc=$rc"; exit $rc; fi
  # a GPU fault reported through a Python exception also exits 1: stop there too
  if grep -q -E "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "$out/step$i.log"; then
    echo "[gpu_steps] stopping: GPU fault in step $i"; exit 3
  fi
done
