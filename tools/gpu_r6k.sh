set -o pipefail
mkdir -p gpurun_out/r6k
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_service.py tests/test_connection_e2e.py -m gpu > gpurun_out/r6k/pytest_service.log 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6k/conn.json 2> gpurun_out/r6k/conn.err
