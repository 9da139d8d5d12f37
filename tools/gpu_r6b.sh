#!/bin/bash
# Round 6 (b): phased launch beside another context's worker (registry counts
# every service-enabled context), the late-follower test, the phased tests,
# the per-k table above k = 16, then a bench run with the beside-service leg.
# Usage: tools/gpu_r6b.sh <tag>
TAG=${1:-r6b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_service.py -m gpu -x -v -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_service.log" 2>&1 &&
tail -3 "$OUT/pytest_service.log" &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-connection --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 python -u -m pytest tests/test_hip_phase.py -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/pytest_phase.log" 2>&1 &&
tail -3 "$OUT/pytest_phase.log" &&
timeout -k 10 600 python -u tools/phase_k_table.py 3 8 10,17,18,20,24,28,32,48,64,128,255 > "$OUT/phase_k_table.txt" 2>&1
rc=$?
tail -16 "$OUT/phase_k_table.txt"
exit $rc
