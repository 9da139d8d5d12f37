mkdir -p gpurun_out
timeout -k 10 300 tools/tune/build/tune_rw 10 5 > gpurun_out/tune_rw_j.txt 2>&1 && \
timeout -k 10 300 tools/tune/build/tune_rw 10 3 5 11 64 400 > gpurun_out/tune_rw_j_small.txt 2>&1
echo rc=$?
