mkdir -p gpurun_out/lat
timeout -k 10 120 tools/tune/build/tune_flush > gpurun_out/lat/tune_flush_pb32.txt 2>&1
echo rc=$?
