mkdir -p gpurun_out/al3
TUNE_RW_BLOCK2=1 TUNE_RW_PALIGN=16 timeout -k 10 300 tools/tune/build/tune_rw 10 5 5 11 64 1287 0 1536 > gpurun_out/al3/block2_a16.txt 2>&1 && tail -30 gpurun_out/al3/block2_a16.txt
