#!/bin/bash
# Round 6 (j): paced native feeder (beside test + bench leg), templated phased
# recover for k = 17-32 (phase tests, per-k table).
TAG=${1:-r6j}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_service.py tests/test_hip_phase.py -m gpu -v -s \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"; grep "abandoned" "$OUT/pytest.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u tools/phase_k_table.py 5 8 17,20,24,26,28,32 > "$OUT/phase_k_table.txt" 2>&1 &&
tail -9 "$OUT/phase_k_table.txt" &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-cpu-baseline --no-ceilings --no-connection > "$OUT/bench.json" 2> "$OUT/bench.err"
rc3=$?
grep -o '"phase_beside_service": {[^}]*}' "$OUT/bench.json"
[ $rc3 -eq 0 ] && exit $rc
exit $rc3
