mkdir -p gpurun_out/r4f && export TMPDIR=/tmp &&
timeout -k 10 240 tools/tune/build/null_phased 10485760 5 3 > gpurun_out/r4f/null_phased.txt 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r4f/bench.json 2> gpurun_out/r4f/bench.err && tail -c 1200 gpurun_out/r4f/bench.json
