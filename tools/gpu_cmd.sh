mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 && \
timeout -k 10 300 tests/cpp/build/bench_connection > gpurun_out/bench_connection.json 2> gpurun_out/bench_connection.err
echo rc=$?
