mkdir -p gpurun_out/p2d
timeout -k 10 300 tools/tune/build/place_2d 5 3 > gpurun_out/p2d/run1.txt 2>&1 && \
timeout -k 10 300 tools/tune/build/place_2d 5 3 > gpurun_out/p2d/run2.txt 2>&1 && \
timeout -k 10 300 tools/tune/build/place_2d 5 3 > gpurun_out/p2d/run3.txt 2>&1
echo rc=$?
