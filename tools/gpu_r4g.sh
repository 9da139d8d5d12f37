#!/bin/bash
# Round-4 GPU session g: the small-batch service (resident worker) -- its
# tests, the mapped / connection tests that now route small batches through
# it, then the connection e2e and host-cost measurements.
TAG=${1:-r4g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_service.py tests/test_hip_mapped.py tests/test_connection_e2e.py tests/test_connection.py > "$OUT/pytest_svc.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_svc.log"; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > "$OUT/conn_e2e.txt" 2>&1 &&
timeout -k 10 200 tools/tune/build/host_cost 64 1024 4096 > "$OUT/host_cost.txt" 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection(cpu=False)))" > "$OUT/connection.txt" 2>&1
