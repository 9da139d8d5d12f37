"""Per-group-size table of the phased fixed-shape kernel (DESIGN.md §4,
VERDICT r3 item 7, r4 item 3): for every k given, 2^20 groups x k x 1350 B,
encode and recover with the register-held phase steps (the product since
round 4) and without them (qfec_debug_phase_regsteps(0): 40 LDS steps per
phase, round 3's kernel for k != 10), alternated round by round in one
process on the same buffers.  The outputs of the two forms are compared
byte for byte, and the round trip (revived row == lost row) is checked.
GPU box; one JSON line per k, then a summary.

  python tools/phase_k_table.py [rounds=3] [reps=8] [k,k,...]

The one-pass kernel (QFEC_ONE_PASS) is timed beside them on the same buffers;
the library's default choice (no test hook) is run once to see which kernel it
picks, and reported as that kernel's column (the same kernel on the same
buffers: a second timing of it only adds noise), with its ratio to the best.  k > 16 has no
register steps (runtime-k body): its two phased columns are the load batch of
32 ("register steps" column) and of 16 ("LDS steps only" column; both set
through qfec_debug_phase_rtbatch), over 2^18 groups above k = 32; the
default column is the library's per-operation choice (phase_rt_batch).
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from libquic_amd import qfec  # noqa: E402

HBM = 8000.0  # GB/s, MI355X_MICROARCH.md


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    L = 1350
    ctx = qfec.Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    out_rows = []
    ks = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 4, 5, 8, 10, 16]
    for k in ks:
        # 2^20 groups up to k = 32; above, 2^18 (>= 8 phases of 40 steps on
        # 256 CUs, 90 GB at k = 255)
        G = 1 << 20 if k <= 32 else 1 << 18
        rows = torch.empty(G * k * L, dtype=torch.uint8, device=dev)
        ctx.synth_fixed(rows, k, L, 0, G, 0x5EED0000 + k)
        miss = torch.from_numpy(
            (np.random.default_rng(k).integers(0, k, G)).astype(np.uint8)).to(dev)
        par = {m: torch.empty(G * L, dtype=torch.uint8, device=dev) for m in (0, 1)}
        out = {m: torch.empty(G * L, dtype=torch.uint8, device=dev) for m in (0, 1)}
        par[2], out[2] = par[0], out[0]  # one-pass writes where LDS-only did (compared below)
        par[3], out[3] = par[2], out[2]
        t = {(m, op): [] for m in (0, 1, 2, 3) for op in ("enc", "rec")}
        phased = {}
        for r in range(rounds):
            for m in (1, 0, 2, 3):  # 1: register steps, 0: LDS steps only, 2: one-pass,
                # 3: the library's default choice (no hook)
                # k > 16 (runtime-k body, no register steps): mode 0 is the
                # load batch of 16, mode 1 the batch of 32 (mode 3: the
                # library's per-op choice, phase_rt_batch)
                ctx.debug_phase_regsteps(m != 0 or k > 16)
                # (k > 16: a nonzero batch forces the runtime-k body, also
                # where k is templated; mode 3, the default, takes neither hook)
                ctx.debug_phase_rtbatch((16 if m == 0 else 32 if m == 1 else 0) if k > 16 else 0)
                # phased forms at every k (the library's default picks one-pass
                # below k = 5 / 8 since round 4, from this very table)
                ctx.debug_phase_min(6 if m in (0, 1) else 0)
                # modes 0 and 1 swap their two output buffers round by round
                # (their A/B is not also an A/B of two DRAM placements)
                bi = (m + r) % 2 if m in (0, 1) else m
                for op in ("enc", "rec"):
                    def run():
                        if op == "enc":
                            ctx.encode(rows, k, L, G, par[bi], one_pass=(m == 2))
                        else:
                            ctx.recover(rows, par[bi], miss, k, L, G, out[bi], one_pass=(m == 2))
                    run()  # warm
                    phased[(m, op)] = ctx.last_fixed_phased()
                    if m == 3 and k <= 16:
                        continue  # the default: which kernel it picks (timed as its column)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(reps):
                        run()
                    e1.record(stream)
                    e1.synchronize()
                    t[(m, op)].append(e0.elapsed_time(e1) / reps / 1e3)
        ctx.debug_phase_regsteps(True)
        ctx.debug_phase_rtbatch(0)
        ctx.debug_phase_min(0)
        ctx.sync()
        torch.cuda.synchronize()
        same = torch.equal(par[0], par[1]) and torch.equal(out[0], out[1])  # one-pass wrote 0 last
        r3 = rows.view(G, k, L)
        trip = torch.equal(r3[torch.arange(G, device=dev), miss.long()], out[1].view(G, L))
        b = G * (k + 1) * L  # encode: k rows read + parity written; recover: k-1 + parity + out
        rec = {"k": k, "groups": G, "L": L, "identical": bool(same), "round_trip": bool(trip),
               "phased": {f"{m}{op}": phased[(m, op)] for (m, op) in phased}}
        for m, tag in ((1, "regsteps"), (0, "lds_only"), (2, "one_pass")):
            for op in ("enc", "rec"):
                s = float(np.median(t[(m, op)]))
                rec[f"{tag}_{op}_us"] = round(s * 1e6, 1)
                rec[f"{tag}_{op}_frac"] = round(b / s / 1e9 / HBM, 4)
        for op in ("enc", "rec"):
            # k <= 16: the library's default IS one of the timed kernels on
            # the same buffers (one-pass, or phased with register steps);
            # k > 16: timed itself (a templated k, round 6, or the runtime-k
            # body with the batch phase_rt_batch picks)
            if k > 16:
                sdef = float(np.median(t[(3, op)]))
                rec[f"default_{op}_frac"] = round(b / sdef / 1e9 / HBM, 4)
                rec[f"default_{op}_is"] = "timed"
            else:
                col = 2 if phased[(3, op)] != 1 else 1
                tag = {1: "regsteps", 2: "one_pass"}[col]
                rec[f"default_{op}_frac"] = rec[f"{tag}_{op}_frac"]
                rec[f"default_{op}_is"] = tag
            best = max(rec[f"regsteps_{op}_frac"], rec[f"lds_only_{op}_frac"],
                       rec[f"one_pass_{op}_frac"], rec[f"default_{op}_frac"])
            rec[f"default_{op}_of_best"] = round(rec[f"default_{op}_frac"] / best, 4)
        print(json.dumps(rec), flush=True)
        out_rows.append(rec)
        del rows, par, out
        torch.cuda.empty_cache()
    print("\n| k | encode: register steps / LDS steps only / one-pass -> default (kernel) | "
          "recover: register steps / LDS steps only / one-pass -> default (kernel) | "
          "default / best of the three, enc / rec |")
    print("|---|---|---|---|")
    for r in out_rows:
        ke = "phased" if r["phased"]["3enc"] == 1 else "one-pass"
        kr = "phased" if r["phased"]["3rec"] == 1 else "one-pass"
        print(f"| {r['k']} | {r['regsteps_enc_frac']:.3f} / {r['lds_only_enc_frac']:.3f} / "
              f"{r['one_pass_enc_frac']:.3f} -> **{r['default_enc_frac']:.3f}** ({ke}) | "
              f"{r['regsteps_rec_frac']:.3f} / {r['lds_only_rec_frac']:.3f} / "
              f"{r['one_pass_rec_frac']:.3f} -> **{r['default_rec_frac']:.3f}** ({kr}) | "
              f"{r['default_enc_of_best']:.3f} / {r['default_rec_of_best']:.3f} |")
    ok = all(r["identical"] and r["round_trip"] for r in out_rows)
    print("all identical and round trips exact:", ok)
    return 0 if ok else 2


if __name__ == "__main__":
    sys.exit(main())
