#!/bin/bash
# what keeps the AEAD kernels' VALU and LDS idle.  Two
# --pmc passes over `bench.py --protect-only` (at most 8 SQ counters each):
# pass A = occupancy and waits (waves resident, wave-cycles, cycles waiting
# for any instruction / for LDS, issue activity), pass B = LDS pipeline
# (bank conflicts, command / data FIFO full, LDS instructions in flight).
# tools/aead_stall.py -> profiles/round5/aead_stall.json.
# Usage: tools/pmc_aead_stall.sh <tag>
TAG=${1:-stall}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_stall_a" -o run -- python bench.py --protect-only > "$OUT/pmc_stall_a.log" 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_stall_b" -o run -- python bench.py --protect-only > "$OUT/pmc_stall_b.log" 2>&1 && \
python tools/aead_stall.py "$OUT" "$OUT/pmc_stall_a.log"
