mkdir -p gpurun_out/rs2
timeout -k 10 300 python -u -m pytest tests/test_hip_phase.py tests/test_hip_fixed.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rs2/pytest.log 2>&1 && tail -3 gpurun_out/rs2/pytest.log &&
timeout -k 10 300 tools/tune/build/tune_phase 5 3 > gpurun_out/rs2/tune_phase_rs2.txt 2>&1 && tail -n 22 gpurun_out/rs2/tune_phase_rs2.txt
