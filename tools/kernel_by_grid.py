"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV.

rocprofv3's --stats averages every dispatch of a kernel name together; the
default bench also runs the same encode/recover kernels on small chunks (the
pinned-host end-to-end leg), so the headline launches (2^20 groups) are
separated here by grid size.  Usage:

    python tools/kernel_by_grid.py gpurun_out/<tag>/prof/run_kernel_trace.csv [out.csv]
"""
import collections
import csv
import statistics
import sys


def summarise(trace_csv):
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        groups[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (name, grid, wg), d in groups.items():
        rows.append({"Name": name, "Grid_Size_X": grid, "Workgroup_Size_X": wg, "Calls": len(d),
                     "AverageNs": round(statistics.mean(d), 1),
                     "MedianNs": statistics.median(d), "MinNs": min(d), "MaxNs": max(d),
                     "TotalNs": sum(d)})
    rows.sort(key=lambda r: -r["TotalNs"])
    return rows


def main():
    rows = summarise(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)


if __name__ == "__main__":
    main()
