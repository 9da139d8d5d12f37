#!/bin/bash
# HBM traffic of the FEC kernels from PMC counters, one counter per pass
# (MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE
# cannot share a pass).  Usage: tools/pmc.sh <tag>
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run \
    -- python bench.py --profile-only --steps 3 --warmup 1 --no-verify > "$OUT/pmc_$C.log" 2>&1
  rc=$?
  echo "[pmc $C] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/parse_prof.py "$OUT"
