"""Compute-side counters of the protection kernels from the two rocprofv3
--pmc passes over `bench.py --protect-only` (tools/pmc_protect.sh).

Writes profiles/protect_insts_latest.json: per kernel, the mean per dispatch
of every counter, the wave-instruction counts per packet (the batch's packet
count from the run's JSON line) and the busy fractions of the CUs' VALU, LDS
and scalar units over the kernel (rocprofv3's VALUBusy: SQ_ACTIVE_INST_VALU /
CU_NUM / max-over-XCDs GRBM_GUI_ACTIVE; likewise LDS) — the compute-roofline
fractions bench.py reports next to the HBM fraction.
Usage: python tools/protect_insts.py <run dir> <bench log>"""
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CU_NUM = 256  # MI355X (MI355X_MICROARCH.md)
N_XCC = 8     # GRBM_GUI_ACTIVE arrives summed over the 8 XCDs; VALUBusy takes its max


def main(d, log):
    line = [l for l in open(log) if l.startswith("{")][-1]
    n = json.loads(line)["protect"]["packets"]
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"qfec::\(anonymous namespace\)::", "", row["Kernel_Name"])
            k = re.sub(r"\(.*", "", k).replace("void ", "").strip()
            vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(
                float(row["Counter_Value"]))
    out = {"packets": n, "source": d, "cu_num": CU_NUM, "kernels": {}}
    for k, cs in vals.items():
        if not any(t in k for t in ("null_", "c20p1305", "aes128gcm")):
            continue
        m = {c: statistics.mean(v) for c, v in cs.items()}
        kd = {"per_dispatch": m,
              "per_packet": {c: v / n for c, v in m.items() if c.startswith("SQ_INSTS_")}}
        g = m.get("GRBM_GUI_ACTIVE")
        if g:
            g /= N_XCC
            for unit in ("VALU", "LDS", "SALU"):
                a = m.get(f"SQ_ACTIVE_INST_{unit}")
                if a is not None:
                    kd[f"{unit.lower()}_busy"] = a / CU_NUM / g
        out["kernels"][k] = kd
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "protect_insts_latest.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
