#!/bin/bash
# Round-4 GPU session b: the phased-copy probe (NULL protection bound), then
# the final tree's evidence set -- GPU tests, smoke, bench, the bench under
# rocprofv3 --kernel-trace --stats, PMC traffic (FETCH_SIZE / WRITE_SIZE, one
# counter per pass) and the protection kernels' compute counters.
# Steps chained with &&: the first failure ends the call.
# Usage: tools/gpu_r4b.sh <tag>
TAG=${1:-r4b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/fused_probe.py > "$OUT/fused_probe.txt" 2>&1 &&
bash tools/gpu_check.sh "$TAG" &&
bash tools/pmc.sh "$TAG" &&
bash tools/pmc_protect.sh "$TAG"
