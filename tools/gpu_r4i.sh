#!/bin/bash
# Round-4 GPU session i: recover register-step variants (tune_phase), then
# the bench with the fused leg ahead of the host-staging leg.
TAG=${1:-r4i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 tools/tune/build/tune_phase 5 3 > "$OUT/tune_phase.txt" 2>&1 && tail -n 24 "$OUT/tune_phase.txt" &&
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && tail -c 1300 "$OUT/bench.json"
