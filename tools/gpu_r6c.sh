#!/bin/bash
# Round 6 (c): runtime-k recover with parity first + compact rows, per-op load
# batch; phase tests, the per-k table above 16, the bench's beside-service leg.
# Usage: tools/gpu_r6c.sh <tag>
TAG=${1:-r6c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_phase.py -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/pytest_phase.log" 2>&1 &&
tail -3 "$OUT/pytest_phase.log" &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-connection --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 600 python -u tools/phase_k_table.py 3 8 10,17,20,24,32,33,48,64,128,255 > "$OUT/phase_k_table.txt" 2>&1
rc=$?
tail -14 "$OUT/phase_k_table.txt"
exit $rc
