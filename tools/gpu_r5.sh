#!/bin/bash
# Round-5 GPU session: the GPU suite, the per-k table (every k templated up to
# 16, the runtime-k body above), then the default bench line.
#   tools/gpu_r5.sh TAG [steps...]   steps: tests ktable bench (default: all)
TAG=${1:-r5a}
shift
STEPS=${*:-tests ktable bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -n 3 "$OUT/pytest_gpu.log" ;;
    ktable)
      timeout -k 10 600 python -u tools/phase_k_table.py 2 5 2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,20,32 \
        > "$OUT/phase_k_table.txt" 2>&1 || { tail -n 30 "$OUT/phase_k_table.txt"; exit 1; }
      tail -n 22 "$OUT/phase_k_table.txt" ;;
    bench)
      timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -n 30 "$OUT/bench.err"; exit 1; }
      tail -c 1500 "$OUT/bench.json" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
