#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 700 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
