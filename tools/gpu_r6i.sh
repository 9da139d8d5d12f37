#!/bin/bash
# Round 6 (i): native service feeder (bench leg + beside test), k = 20
# templated for the phased kernel (phase tests, per-k table at 17 / 20 / 24).
TAG=${1:-r6i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_service.py tests/test_hip_phase.py -m gpu -v -s \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"; grep "abandoned" "$OUT/pytest.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/phase_k_table.py 5 8 16,17,20,24 > "$OUT/phase_k_table.txt" 2>&1 &&
tail -8 "$OUT/phase_k_table.txt" &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-ragged --no-protect --no-entropy \
  --no-fused --no-e2e --no-cpu-baseline --no-ceilings --no-connection > "$OUT/bench.json" 2> "$OUT/bench.err"
rc3=$?
grep -o '"phase_beside_service": {[^}]*}' "$OUT/bench.json"
[ $rc3 -eq 0 ] && exit $rc
exit $rc3
