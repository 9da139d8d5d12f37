mkdir -p gpurun_out/r1w; timeout -k 10 300 tools/tune/build/tune_ragged 10 5 > gpurun_out/r1w/tune_ragged.txt 2>&1; rc=$?; cat gpurun_out/r1w/tune_ragged.txt; exit $rc
