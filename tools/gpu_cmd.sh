mkdir -p gpurun_out/rc4
timeout -k 10 180 tools/tune/build/tune_rchunk 10 4 > gpurun_out/rc4/tune_rchunk.txt 2>&1
rc=$?; echo rc=$rc; cat gpurun_out/rc4/tune_rchunk.txt; exit $rc
