#!/bin/bash
# Round 6 (a): service protocol (announced split jobs, follower hold test,
# phased launch beside another context's fed worker), runtime-k phased body
# parity, then the per-k table above k = 16.  Steps chained: the first
# failure ends the call.
# Usage: tools/gpu_r6a.sh <tag>
TAG=${1:-r6a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_service.py tests/test_hip_mapped.py -m gpu -x -v -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_service.log" 2>&1 &&
tail -3 "$OUT/pytest_service.log" &&
timeout -k 10 600 python -u -m pytest tests/test_hip_phase.py -m gpu -x -v -s -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/pytest_phase.log" 2>&1 &&
tail -3 "$OUT/pytest_phase.log" &&
timeout -k 10 900 python -u tools/phase_k_table.py 3 8 10,17,18,20,24,28,32,48,64,128,255 > "$OUT/phase_k_table.txt" 2>&1
rc=$?
tail -16 "$OUT/phase_k_table.txt"
exit $rc
