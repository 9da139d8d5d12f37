set -o pipefail
mkdir -p gpurun_out/r6p
timeout -k 10 300 ./tools/probe_bin/tune_rblock 10 5 16 1536 3 > gpurun_out/r6p/tune_rblock_cache_a16.txt 2>&1 &&
timeout -k 10 300 ./tools/probe_bin/tune_rblock 10 5 1 1452 3 > gpurun_out/r6p/tune_rblock_cache_a1.txt 2>&1
