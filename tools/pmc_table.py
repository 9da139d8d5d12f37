"""Per-kernel PMC table from rocprofv3 --pmc passes (one sub-directory per
pass under DIR, each holding *counter_collection.csv): mean value per dispatch
of every counter, per kernel name.  Usage: python tools/pmc_table.py DIR [filter]"""
import csv
import glob
import os
import re
import statistics
import sys


def short(name):
    name = re.sub(r"qfec::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(qfec::RaggedArgs\)|\(qfec::FixedArgs.*\)", "", name)
    return name.strip()


def main(d, filt=""):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if filt and filt not in k:
                    continue
                vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(
                    float(row["Counter_Value"]))
    for k in sorted(vals):
        cs = vals[k]
        print(k)
        for c in sorted(cs):
            print(f"    {c:36s} {statistics.mean(cs[c]):14.4g}  (n={len(cs[c])})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
