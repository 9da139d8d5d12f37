#!/bin/bash
# Round-5: the ragged phased prototype (tools/tune/tune_rphase.hip) on the
# configs[3] batch, arena layout (16-B aligned payloads, 1536-B slots) and
# byte-packed (1452-B slots).
TAG=${1:-rp1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 tools/tune/build/tune_rphase 5 3 16 1536 > "$OUT/rphase_a16.txt" 2>&1; rc=$?
cat "$OUT/rphase_a16.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/tune/build/tune_rphase 5 3 1 1452 > "$OUT/rphase_packed.txt" 2>&1; rc=$?
tail -n 14 "$OUT/rphase_packed.txt"
exit $rc
