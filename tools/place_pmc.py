"""Per-launch table of tools/tune/place_pmc runs: every fixed-encode dispatch
of each rocprofv3 --pmc pass, its destination and HIP-event time (from the
program's own output) and that pass's counters.  Usage:
    python tools/place_pmc.py gpurun_out/ppmc
(the directory holds pN.txt + pN/run_counter_collection.csv per pass)."""
import csv
import glob
import os
import re
import sys


def main(d):
    for txt in sorted(glob.glob(os.path.join(d, "p*.txt"))):
        p = os.path.splitext(os.path.basename(txt))[0]
        launches = [re.match(r"dispatch (\d+) dst (\S+) rep (\d+) us ([\d.]+) frac ([\d.]+)", l)
                    for l in open(txt)]
        launches = [m.groups() for m in launches if m]
        rows = {}
        for f in glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "fixed_xor_kernel" not in r["Kernel_Name"]:
                    continue
                rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(
                    r["Counter_Value"])
        ids = sorted(rows)
        if not ids:
            continue
        names = sorted(rows[ids[0]])
        print(f"== {p}: " + "  ".join(names))
        for (_, dst, rep, us, frac), i in zip(launches, ids):
            vals = "  ".join(f"{rows[i][n]:.4g}" for n in names)
            print(f"{dst:7s} {rep} {float(us):7.1f} us {frac}  {vals}")


if __name__ == "__main__":
    main(sys.argv[1])
