set -o pipefail
mkdir -p gpurun_out/r6t
timeout -k 10 400 python -u tools/svc_trace.py 200 1,4,8,9,16,32,48,64 30 > gpurun_out/r6t/svc_trace_n.txt 2>&1
