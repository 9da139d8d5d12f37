#!/bin/bash
# Round-4 GPU session c: GPU tests, then the measurements gpu_r4.sh did not
# reach (host cost, PCIe duplex, connection e2e), the phased-copy probe and
# the bench.  Steps chained with &&: the first failure ends the call.
# Usage: tools/gpu_r4c.sh <tag>
TAG=${1:-r4c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/pytest_gpu.log" 2>&1 && tail -2 "$OUT/pytest_gpu.log" &&
timeout -k 10 200 tools/tune/build/host_cost 64 1024 4096 16384 > "$OUT/host_cost.txt" 2>&1 &&
timeout -k 10 120 tools/tune/build/pcie_duplex 1024 7 > "$OUT/pcie_duplex.txt" 2>&1 &&
HSA_ENABLE_SDMA=0 timeout -k 10 120 tools/tune/build/pcie_duplex 1024 7 > "$OUT/pcie_duplex_nosdma.txt" 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > "$OUT/conn_e2e.txt" 2>&1 &&
timeout -k 10 240 tools/tune/build/phased_copy 4096 5 3 > "$OUT/phased_copy.txt" 2>&1 &&
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && tail -c 1500 "$OUT/bench.json"
