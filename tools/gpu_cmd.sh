mkdir -p gpurun_out/win
export TUNE_RW_PALIGN=16
TUNE_RW_WINAL=1 timeout -k 10 200 tools/tune/build/tune_rw 10 5 5 11 64 1287 0 1536 > gpurun_out/win/winal.txt 2>&1; rc=$?; tail -n 14 gpurun_out/win/winal.txt; exit $rc
