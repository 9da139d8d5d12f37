#!/bin/bash
# One GPU iteration: parity tests, the ragged-variant stress, the ragged A/B
# timing and a device-only bench line.  Stops at the first failing step.
# Usage: tools/gpu_iter.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-iter}
mkdir -p "$OUT"
step() {  # $1 = name, $2 = timeout, rest = command; output to $OUT/$1.log
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -25 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
step ragged_variants 300 tools/debug/build/ragged_variants 6
step tune_ragged 300 tools/tune/build/tune_ragged 10 5
step bench 600 python bench.py --no-cpu-baseline --no-e2e
