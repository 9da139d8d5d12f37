#!/bin/bash
# Round 6 (f): service tests (quiet-context grid with the registry's view),
# the end-to-end service trace (1 / 64 groups x assembly gaps), the bench's
# connection legs.
TAG=${1:-r6f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_service.py -m gpu -v -s \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_service.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_service.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/svc_trace.py 300 > "$OUT/svc_trace.txt" 2>&1 &&
cat "$OUT/svc_trace.txt" &&
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-cpu-baseline --no-ceilings --no-beside-service > "$OUT/bench.json" 2> "$OUT/bench.err"
rc3=$?
grep -o '"connection": {.\{0,900\}' "$OUT/bench.json" | head -c 1200
[ $rc3 -eq 0 ] && exit $rc
exit $rc3
