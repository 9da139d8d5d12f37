set -o pipefail
mkdir -p gpurun_out/r6n
timeout -k 10 400 python -u -m pytest -v -s -x --timeout 120 --timeout-method thread tests/test_hip_service.py tests/test_connection_e2e.py tests/test_hip_mapped.py -m gpu > gpurun_out/r6n/pytest_service.log 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection()))" > gpurun_out/r6n/conn_legs1.json 2> gpurun_out/r6n/conn_legs1.err &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection()))" > gpurun_out/r6n/conn_legs2.json 2> gpurun_out/r6n/conn_legs2.err &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6n/conn_e2e.json 2> gpurun_out/r6n/conn_e2e.err
