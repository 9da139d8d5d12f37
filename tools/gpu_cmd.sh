mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/ab/tests.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw 10 5 > gpurun_out/ab/new1.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw_old 10 5 > gpurun_out/ab/old1.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw 10 5 > gpurun_out/ab/new2.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw_old 10 5 > gpurun_out/ab/old2.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw 10 3 5 11 64 400 > gpurun_out/ab/new_small.txt 2>&1 && \
timeout -k 10 200 tools/tune/build/tune_rw_old 10 3 5 11 64 400 > gpurun_out/ab/old_small.txt 2>&1
echo rc=$?
