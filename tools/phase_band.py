"""The phased kernel's lower edge: fixed-shape encode and
recover at k = 10, L = 1350 from 16K to 1M groups, the one-pass kernel
(QFEC_ONE_PASS) against the phased one forced at every size
(qfec_debug_phase_min(ctx, 1)), interleaved, device-resident, HIP events on
the context's stream; parity / revived rows of the two compared.  Output: one
line per size and a JSON summary (fraction of 8 TB/s on the algorithmic
bytes).  Usage on the GPU box: python tools/phase_band.py [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libquic_amd import qfec  # noqa: E402

K, L, SEED = 10, 1350, 0x51554943
SIZES = [16384, 32768, 65536, 131072, 196608, 262144, 393216, 524288, 1048576]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    ctx = qfec.Context(0)
    gmax = SIZES[-1]
    rows = torch.empty(gmax * K * L, dtype=torch.uint8, device=dev)
    ctx.synth_fixed(rows, K, L, 0, gmax, SEED)
    par = {m: torch.empty(gmax * L, dtype=torch.uint8, device=dev) for m in ("one", "ph")}
    out = {m: torch.empty(gmax * L, dtype=torch.uint8, device=dev) for m in ("one", "ph")}
    missing = (torch.arange(gmax, device=dev) % K).to(torch.uint8)
    ctx.sync()
    s = torch.cuda.Stream()
    ctx.set_stream(s)  # events on the kernels' own stream
    res = []
    for G in SIZES:
        t = {}
        for m in ("one", "ph"):
            t[m] = {"enc": [], "rec": []}
        for r in range(reps + 1):
            for m in ("one", "ph"):
                ctx.debug_phase_min(1 if m == "ph" else 0)
                for op in ("enc", "rec"):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    if op == "enc":
                        ctx.encode(rows, K, L, G, par[m], one_pass=(m == "one"))
                    else:
                        ctx.recover(rows, par["one"], missing, K, L, G, out[m], one_pass=(m == "one"))
                    e1.record(s)
                    e1.synchronize()
                    if r:
                        t[m][op].append(e0.elapsed_time(e1))
        ctx.debug_phase_min(0)
        same_p = torch.equal(par["one"][:G * L], par["ph"][:G * L])
        same_r = torch.equal(out["one"][:G * L], out["ph"][:G * L])
        eb = G * (K * L + L)          # encode: k rows read, parity written
        rb = G * (K * L + L)          # recover: k-1 rows + parity read, 1 row written
        row = {"groups": G, "parity_identical": same_p, "revived_identical": same_r}
        for m in ("one", "ph"):
            for op, b in (("enc", eb), ("rec", rb)):
                ms = sorted(t[m][op])[len(t[m][op]) // 2]
                row[f"{m}_{op}_ms"] = round(ms, 4)
                row[f"{m}_{op}_frac"] = round(b / (ms * 1e-3) / 8e12, 3)
        res.append(row)
        print(f"G={G:8d}  encode one-pass {row['one_enc_frac']:.3f} phased {row['ph_enc_frac']:.3f}"
              f"   recover one-pass {row['one_rec_frac']:.3f} phased {row['ph_rec_frac']:.3f}"
              f"   identical {same_p and same_r}", flush=True)
    print(json.dumps({"phase_band": res, "abandons": ctx.phase_abandons()}))


if __name__ == "__main__":
    main()
