mkdir -p gpurun_out/lo
timeout -k 10 200 tools/tune/build/tune_rw 10 5 > gpurun_out/lo/tune_rw_lo.txt 2>&1
timeout -k 10 120 tools/tune/build/place_pmc 2 > gpurun_out/lo/fixed.txt 2>&1
echo rc=$?
