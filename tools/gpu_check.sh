#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / timeout (rc other than 0 or 1).
# Usage: tools/gpu_check.sh [tag]
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ok_or_fail() {  # $1 = rc, $2 = step name
  echo "[$2] rc=$1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "[$2] fatal rc=$1, stopping"; exit "$1"; fi
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
ok_or_fail $? pytest_gpu
tail -5 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok_or_fail $? smoke
cat "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
ok_or_fail $? bench
cat "$OUT/bench.json"
# the same default bench command under the profiler: its JSON line and the
# kernel stats come from one process (bench_prof.json)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
  -- python bench.py > "$OUT/bench_prof.json" 2> "$OUT/prof.log"
ok_or_fail $? rocprof_stats
find "$OUT/prof" -name '*stats*' | head
python tools/kernel_by_grid.py "$OUT/prof/run_kernel_trace.csv" "$OUT/prof/kernel_by_grid.csv"
