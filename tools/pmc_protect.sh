#!/bin/bash
# Compute-side counters of the packet-protection kernels for bench.py's
# protect compute-roofline fractions: pass 1 = wave-instruction counts (VALU /
# LDS / scalar / vector memory), pass 2 = the cycles the CUs' VALU / LDS /
# units were busy (rocprofv3's VALUBusy definition:
# SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE), both over
# `bench.py --protect-only`; tools/protect_insts.py ->
# profiles/protect_insts_latest.json.
# Usage: tools/pmc_protect.sh <tag>
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/pmc_protect" -o run -- python bench.py --protect-only > "$OUT/pmc_protect.log" 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_protect_busy" -o run -- python bench.py --protect-only > "$OUT/pmc_protect_busy.log" 2>&1 && \
python tools/protect_insts.py "$OUT" "$OUT/pmc_protect.log"
