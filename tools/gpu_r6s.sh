set -o pipefail
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u -m pytest -v -s -x --timeout 120 --timeout-method thread tests/test_hip_service.py tests/test_connection_e2e.py tests/test_hip_mapped.py -m gpu > gpurun_out/r6s/pytest_service.log 2>&1
