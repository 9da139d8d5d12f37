set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 120 python -u tools/debug_hold2.py > gpurun_out/r6v/debug_hold2.txt 2>&1
