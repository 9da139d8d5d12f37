set -o pipefail
mkdir -p gpurun_out/r6r
timeout -k 10 400 python -u -m pytest -v -s -x --timeout 120 --timeout-method thread tests/test_hip_service.py tests/test_connection_e2e.py -m gpu > gpurun_out/r6r/pytest_service.log 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection()))" > gpurun_out/r6r/conn_legs.json 2> gpurun_out/r6r/conn_legs.err
