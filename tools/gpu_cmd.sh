mkdir -p gpurun_out/reg
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_mapped.py tests/test_abi.py > gpurun_out/reg/tests.txt 2>&1
echo rc=$?
