#!/bin/bash
# Round-6 final-tree evidence (tools/gpu_r5final.sh: GPU tests, smoke, bench,
# rocprofv3 kernel stats, PMC traffic, protection counters), then the VRAM
# ring feasibility probe (last: it touches device memory from the host).
TAG=${1:-r6fin}
bash tools/gpu_r5final.sh "$TAG" || exit $?
mkdir -p "gpurun_out/$TAG"
timeout -k 10 120 tools/probe_bin/probe_vram_host 2000 > "gpurun_out/$TAG/probe_vram_host.txt" 2>&1
rc=$?
cat "gpurun_out/$TAG/probe_vram_host.txt"
exit $rc
