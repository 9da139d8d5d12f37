set -o pipefail
mkdir -p gpurun_out/r6o
timeout -k 10 300 python -u tools/svc_trace.py 300 > gpurun_out/r6o/svc_trace.txt 2>&1 &&
timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection()))" > gpurun_out/r6o/conn_legs.json 2> gpurun_out/r6o/conn_legs.err &&
QFEC_SVC_RESIDENT_US=1000000000 timeout -k 10 300 python -u -c "import bench, json; print(json.dumps(bench.bench_connection()))" > gpurun_out/r6o/conn_legs_norot.json 2> gpurun_out/r6o/conn_legs_norot.err
