mkdir -p gpurun_out/cpol
timeout -k 10 400 tools/tune/build/place_cpol 5 3 > gpurun_out/cpol/place_cpol.txt 2>&1
echo rc=$?
