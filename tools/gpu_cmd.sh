mkdir -p gpurun_out/rz
export TUNE_RW_PALIGN=16
B=tools/tune/build
TUNE_RW_BLOCKZ=1 timeout -k 10 120 $B/tune_rw 10 5 5 11 64 1287 0 1536 > gpurun_out/rz/blockz.txt 2>&1 && tail -n 14 gpurun_out/rz/blockz.txt &&
TUNE_RW_BLOCKO=1 timeout -k 10 120 $B/tune_rw 10 5 5 11 64 1287 0 1536 > gpurun_out/rz/blocko.txt 2>&1 && tail -n 16 gpurun_out/rz/blocko.txt
