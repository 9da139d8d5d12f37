set -o pipefail
mkdir -p gpurun_out/r6l
timeout -k 10 60 ./tools/probe_bin/tune_apicost > gpurun_out/r6l/apicost.txt 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6l/conn_default.json 2> gpurun_out/r6l/conn_default.err &&
QFEC_SVC_RESIDENT_US=1000000000 timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6l/conn_norot.json 2> gpurun_out/r6l/conn_norot.err &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection_e2e()))" > gpurun_out/r6l/conn_default2.json 2> gpurun_out/r6l/conn_default2.err
