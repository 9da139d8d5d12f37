#!/bin/bash
# Round 6 (e): service tests (quiet-context grid), bitsliced AES probe, ragged
# 2x2 diag (tail logic x stores), bench beside-service leg with spin stamps.
# A failing test (rc 1) does not stop the later steps; any other failure does.
TAG=${1:-r6e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_service.py -m gpu -v -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_service.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_service.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 tools/tune/build/tune_aes_bitslice $((1<<20)) 5 3 > "$OUT/tune_aes_bitslice.txt" 2>&1
rc2=$?
cat "$OUT/tune_aes_bitslice.txt"
[ $rc2 -le 2 ] || exit $rc2
timeout -k 10 300 tools/tune/build/tune_rblock 10 5 16 1536 1 > "$OUT/tune_rblock_diag.txt" 2>&1 &&
tail -14 "$OUT/tune_rblock_diag.txt" &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-cpu-baseline --no-ceilings --no-connection > "$OUT/bench.json" 2> "$OUT/bench.err" &&
grep -o '"phase_beside_service": {[^}]*}' "$OUT/bench.json"
rc3=$?
[ $rc3 -eq 0 ] && exit $rc
exit $rc3
