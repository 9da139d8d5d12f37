mkdir -p gpurun_out
timeout -k 10 300 tools/tune/build/tune_rw 2 1 > gpurun_out/tune_rw_i.txt 2>&1
echo rc=$?
