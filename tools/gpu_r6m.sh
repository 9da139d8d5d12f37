set -o pipefail
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6m/pytest_gpu.log 2>&1 &&
timeout -k 10 60 ./tools/probe_bin/svc_host_cost 5 > gpurun_out/r6m/svc_host_cost.txt 2>&1 && timeout -k 10 60 ./tools/probe_bin/svc_host_cost 20 >> gpurun_out/r6m/svc_host_cost.txt 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6m/conn1.json 2> gpurun_out/r6m/conn1.err &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6m/conn2.json 2> gpurun_out/r6m/conn2.err
