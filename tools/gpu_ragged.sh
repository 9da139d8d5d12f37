#!/bin/bash
# Ragged path on the GPU: all parity tests, the variant stress and the A/B
# timing.  Stops at the first failing step.  Usage: tools/gpu_ragged.sh <tag>
OUT=gpurun_out/${1:-rg}
mkdir -p "$OUT"
step() {  # $1 = name, $2 = timeout, rest = command
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -30 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
step ragged_variants 300 tools/debug/build/ragged_variants 6
step tune_multi 300 tools/tune/build/tune_multi 10 5
