#!/bin/bash
# Round 6 (d): service (quiet-stretch poll, warm after small turns), mapped and
# connection tests; phase tests; phased grid-size A/B; per-k table (5 rounds,
# default reported as its column); bench connection legs.
# Usage: tools/gpu_r6d.sh <tag>
TAG=${1:-r6d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_service.py tests/test_hip_mapped.py \
  tests/test_connection_e2e.py tests/test_hip_phase.py -m gpu -x -v -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
tail -3 "$OUT/pytest.log" &&
timeout -k 10 300 python -u tools/phase_reserve_ab.py 6 5 > "$OUT/phase_reserve_ab.txt" 2>&1 &&
cat "$OUT/phase_reserve_ab.txt" &&
timeout -k 10 600 python -u tools/phase_k_table.py 5 8 10,17,20,24,32,48,64,128,255 > "$OUT/phase_k_table.txt" 2>&1 &&
tail -13 "$OUT/phase_k_table.txt" &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-cpu-baseline --no-ceilings > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 tools/tune/build/tune_rblock 10 4 16 1536 1 > "$OUT/tune_rblock_diag.txt" 2>&1
tail -12 "$OUT/tune_rblock_diag.txt" &&
timeout -k 10 120 tools/tune/build/tune_hostbw 200 > "$OUT/tune_hostbw.txt" 2>&1
rc=$?
cat "$OUT/tune_hostbw.txt"
exit $rc
