mkdir -p gpurun_out/pl
timeout -k 10 300 tools/tune/build/tune_rw 10 5 > gpurun_out/pl/tune_rw_pl.txt 2>&1 && \
timeout -k 10 300 tools/tune/build/tune_rw 10 5 5 11 64 400 > gpurun_out/pl/tune_rw_pl_small.txt 2>&1
echo rc=$?
