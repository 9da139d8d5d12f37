set -o pipefail
mkdir -p gpurun_out/r6q
timeout -k 10 300 ./tools/probe_bin/tune_rblock 10 5 16 1536 4 > gpurun_out/r6q/tune_rblock_pol_a16.txt 2>&1
