#!/bin/bash
# Round 5: the static-window ragged phased prototype (tools/tune/tune_rpw.hip)
# on configs[3], arena layout (16-B aligned payloads, 1536-B slots), then
# byte-packed (1452-B slots).
TAG=${1:-rpw1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 tools/tune/build/tune_rpw 5 3 16 1536 > "$OUT/rpw_a16.txt" 2>&1; rc=$?
cat "$OUT/rpw_a16.txt"
[ $rc -eq 0 ] || exit $rc
if [ "${2:-}" = packed ]; then
  timeout -k 10 300 tools/tune/build/tune_rpw 5 3 1 1452 > "$OUT/rpw_packed.txt" 2>&1; rc=$?
  tail -n 14 "$OUT/rpw_packed.txt"
fi
exit $rc
