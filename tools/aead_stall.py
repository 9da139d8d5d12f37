"""the AEAD (and NULL) kernels' stall picture from the two
--pmc passes of tools/pmc_aead_stall.sh, beside the instruction counts of
profiles/protect_insts_latest.json.

Per kernel (mean per dispatch): waves resident per SIMD (SQ_LEVEL_WAVES /
SQ_BUSY_CYCLES / 4 SIMDs... as rocprofv3's occupancy), the fraction of wave
cycles a wave waits for anything / for LDS data (SQ_WAIT_ANY, SQ_WAIT_INST_LDS
over SQ_WAVE_CYCLES; all three count quad-cycles, MI355X_MICROARCH.md), the
LDS bank-conflict cycles per LDS instruction, and the VALU / LDS issue
fractions against the CU's issue ceilings (MI355X_MICROARCH.md: SIMD-32, a
wave64 VALU instruction issues in 2 cycles -> 2 wave-instructions per CU per
cycle; ds_read_b32 of 64 lanes = 256 B at 128 B per cycle per CU -> 0.5 per
CU per cycle) over the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs).
Usage: python tools/aead_stall.py <run dir> <bench log>"""
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CU_NUM = 256
N_XCC = 8


def main(d, log):
    vals = {}
    for f in glob.glob(os.path.join(d, "pmc_stall_*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"qfec::\(anonymous namespace\)::", "", row["Kernel_Name"])
            k = re.sub(r"\(.*", "", k).replace("void ", "").strip()
            vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    insts = {}
    p = os.path.join(ROOT, "profiles", "protect_insts_latest.json")
    if os.path.exists(p):
        insts = json.load(open(p)).get("kernels", {})
    out = {"source": d, "cu_num": CU_NUM, "kernels": {}}
    for k, cs in vals.items():
        if not any(t in k for t in ("null_", "c20p1305", "aes128gcm")):
            continue
        m = {c: statistics.mean(v) for c, v in cs.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / N_XCC
        kd = {"per_dispatch": m}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            kd["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0.0) / wc
            kd["wait_inst_any_frac"] = m.get("SQ_WAIT_INST_ANY", 0.0) / wc
            kd["wait_lds_frac"] = m.get("SQ_WAIT_INST_LDS", 0.0) / wc
            kd["active_any_frac"] = m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
        if cyc and m.get("SQ_WAVE_CYCLES"):
            # quad-cycles of resident waves over the kernel's cycles: waves per CU
            kd["waves_per_simd"] = 4.0 * m["SQ_WAVE_CYCLES"] / cyc / CU_NUM / 4.0
        if m.get("SQ_INSTS_LDS"):
            kd["bank_conflict_cycles_per_lds_inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
        ins = insts.get(k, {}).get("per_dispatch", {})
        if cyc and ins.get("SQ_INSTS_VALU"):
            kd["valu_issue_frac"] = ins["SQ_INSTS_VALU"] / CU_NUM / cyc / 2.0
        if cyc and ins.get("SQ_INSTS_LDS"):
            kd["lds_issue_frac"] = ins["SQ_INSTS_LDS"] / CU_NUM / cyc / 0.5
        out["kernels"][k] = kd
    os.makedirs(os.path.join(ROOT, "profiles", "round5"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "round5", "aead_stall.json"), "w") as f:
        json.dump(out, f, indent=1)
    for k, kd in out["kernels"].items():
        print(k, {x: round(v, 3) for x, v in kd.items() if x != "per_dispatch"})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
