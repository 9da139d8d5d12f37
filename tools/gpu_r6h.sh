#!/bin/bash
# Round 6 (h): ragged band table (block kernel vs two groups per wave by group
# shape), then the ragged / mapped GPU tests with the shape-aware choice.
TAG=${1:-r6h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/ragged_band.txt"
for shape in "5 15 64 1350" "5 15 64 900" "5 15 64 700" "5 15 64 463" "2 4 64 1350" \
             "2 6 64 1350" "3 8 64 1350" "4 10 64 1350" "20 40 64 1350" "1 1 64 1350"; do
  for lay in "16 1536" "1 1452"; do
    echo "== shape k/len $shape, layout (align, slot) $lay" >> "$OUT/ragged_band.txt"
    timeout -k 10 120 tools/tune/build/tune_rblock 10 3 $lay 2 $shape >> "$OUT/ragged_band.txt" 2>&1 || exit $?
  done
done
grep -E "^==|groups, k|median" "$OUT/ragged_band.txt"
timeout -k 10 600 python -u -m pytest tests/test_hip_ragged.py tests/test_hip_mapped.py -m gpu -v \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_ragged.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_ragged.log"
exit $rc
