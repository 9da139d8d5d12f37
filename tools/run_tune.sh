#!/bin/bash
# Ragged kernel: variant correctness stress, then A/B timing.  Usage: tools/run_tune.sh <tag>
OUT=gpurun_out/${1:-tune}
mkdir -p "$OUT"
timeout -k 10 300 tools/debug/build/ragged_variants 3 > "$OUT/ragged_variants.txt" 2>&1; rc=$?; cat "$OUT/ragged_variants.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/tune/build/tune_ragged 10 5 > "$OUT/tune_ragged.txt" 2>&1; rc=$?; cat "$OUT/tune_ragged.txt"; exit $rc
