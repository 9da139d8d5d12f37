set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_hip_service.py tests/test_connection_e2e.py tests/test_hip_mapped.py -m gpu > gpurun_out/r6w/pytest_service.log 2>&1 &&
timeout -k 10 400 python -u tools/svc_trace.py 200 1,2,3,4,8 30 > gpurun_out/r6w/svc_trace_n.txt 2>&1
