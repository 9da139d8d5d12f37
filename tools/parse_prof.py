"""Summarise rocprofv3 outputs of a gpu run directory into profiles/.

* kernel stats (--kernel-trace --stats): copied as-is.
* PMC passes (tools/pmc.sh): FETCH_SIZE / WRITE_SIZE per dispatch of the
  fixed-shape encode/recover kernels, in bytes per launch.  Corrections per
  MI355X_MICROARCH.md §HBM: the counters are in KiB; on gfx950 FETCH_SIZE
  reports 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read, so
  it is doubled; WRITE_SIZE is exact for 16-B streaming stores.
Writes profiles/traffic_latest.json (read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kind(name):
    """fixed_xor_kernel<K, RECOVER, NT, SM> / phase_xor_kernel<K, RECOVER, ...> (the
    product's fixed-shape kernels: one-pass and phased) / ragged_block_kernel<RECOVER, ...> (round 3; ragged_multi_kernel before)."""
    m = re.search(r"(?:fixed|phase)_xor_kernel<(-?\d+), (true|false)", name)
    if m:
        return "recover" if m.group(2) == "true" else "encode"
    m = re.search(r"ragged_(?:multi|xor|block)_kernel<(true|false)", name)
    if m:
        return "ragged_recover" if m.group(1) == "true" else "ragged_encode"
    return None


KERNELS = {}


def pmc(run_dir, counter):
    files = glob.glob(os.path.join(run_dir, f"pmc_{counter}", "**", "*counter_collection.csv"),
                      recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = kind(row.get("Kernel_Name", ""))
                if k:
                    vals.setdefault(k, []).append(float(row["Counter_Value"]))
                    kn = re.search(r"(\w+_kernel<[^()]*>)", row.get("Kernel_Name", ""))
                    KERNELS.setdefault(k, set()).add(kn.group(1) if kn else row.get("Kernel_Name", ""))
    return vals


def main(run_dir, groups=1 << 20, k=10, L=1350, layout=None):
    fetch = pmc(run_dir, "FETCH_SIZE")
    write = pmc(run_dir, "WRITE_SIZE")
    out = {"groups": groups, "k": k, "L": L, "source": run_dir,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on wide streaming reads); "
                         "WRITE_SIZE KiB x1024"}
    alg = groups * (k * L + L)
    for kd in ("encode", "recover"):
        if kd in fetch and kd in write:
            f = statistics.median(fetch[kd]) * 1024 * 2
            w = statistics.median(write[kd]) * 1024
            out[f"{kd}_fetch_bytes"] = f
            out[f"{kd}_write_bytes"] = w
            out[f"{kd}_hbm_bytes_per_launch"] = f + w
            out[f"{kd}_traffic_over_algorithmic"] = (f + w) / alg
    # the ragged batch of bench.py (configs[3]); its launches at the batch's
    # full size are the larger ones (the pinned-host / connection legs are not
    # in a --profile-only run)
    if "ragged_encode" in fetch and "ragged_encode" in write:
        sys.path.insert(0, ROOT)
        from bench import ragged_alg_bytes, ragged_layout_tag
        rg = 1 << 20
        alg_e, alg_r = ragged_alg_bytes(rg)
        out["ragged_groups"] = rg
        # the --profile-only leg's layout (bench.py's default unless given)
        out["ragged_layout"] = layout or ragged_layout_tag()
        for kd, alg in (("encode", alg_e), ("recover", alg_r)):
            f_, w_ = fetch.get(f"ragged_{kd}"), write.get(f"ragged_{kd}")
            if f_ and w_:
                f = max(f_) * 1024 * 2
                w = max(w_) * 1024
                out[f"ragged_{kd}_fetch_bytes"] = f
                out[f"ragged_{kd}_write_bytes"] = w
                out[f"ragged_{kd}_algorithmic_bytes"] = alg
                out[f"ragged_{kd}_traffic_over_algorithmic"] = (f + w) / alg
    out["kernels"] = {k: sorted(v) for k, v in KERNELS.items()}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    path = os.path.join(ROOT, "profiles", "traffic_latest.json")
    # per-layout ragged ratios: this run's layout replaces its own entry, the
    # other layouts' entries (earlier runs) are kept with their source
    by = {}
    if os.path.exists(path):
        with open(path) as fh:
            by = json.load(fh).get("ragged_by_layout", {})
    if "ragged_layout" in out:
        by[out["ragged_layout"]] = {
            "encode": out.get("ragged_encode_traffic_over_algorithmic"),
            "recover": out.get("ragged_recover_traffic_over_algorithmic"),
            "source": os.path.basename(os.path.normpath(run_dir))}
    out["ragged_by_layout"] = by
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], layout=sys.argv[2] if len(sys.argv) > 2 else None)
