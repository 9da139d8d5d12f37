#!/bin/bash
# Round 6: runtime-k phased body (load batch 32) -- parity tests for k > 16,
# then the per-k table (tools/phase_k_table.py) above k = 16 and controls.
# Usage: tools/gpu_r6k.sh <tag>
TAG=${1:-r6a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_phase.py -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "runtime_k or vs_one_pass or choice" > "$OUT/pytest_phase.log" 2>&1 &&
tail -3 "$OUT/pytest_phase.log" &&
timeout -k 10 900 python -u tools/phase_k_table.py 3 8 10,17,18,20,24,28,32,48,64,128,255 > "$OUT/phase_k_table.txt" 2>&1
rc=$?
tail -16 "$OUT/phase_k_table.txt"
exit $rc
