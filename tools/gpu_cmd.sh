mkdir -p gpurun_out/r3b
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -v --timeout 180 --timeout-method thread -m gpu tests/test_connection_e2e.py tests/test_integration.py tests/test_hip_mapped.py tests/test_hip_phase.py tests/test_connection.py tests/test_dist.py > gpurun_out/r3b/tests.txt 2>&1
rc=$?; echo rc=$rc; tail -15 gpurun_out/r3b/tests.txt; exit $rc
