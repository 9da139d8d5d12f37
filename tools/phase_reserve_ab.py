"""A/B of the phased grid size (round 6): the headline
batch (2^20 groups x 10 x 1350 B) encoded and recovered with the phased
kernel on every CU, and with 8 / 16 CUs left out of its grid
(qfec_debug_phase_reserve -- what a phased launch does while other contexts'
small-batch workers hold CUs), interleaved round by round in one process on
the same buffers; outputs compared byte for byte.  GPU box.

  python tools/phase_reserve_ab.py [rounds=6] [reps=5]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from libquic_amd import qfec  # noqa: E402

HBM = 8000.0


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    k, L, G = 10, 1350, 1 << 20
    dev = torch.device("cuda:0")
    ctx = qfec.Context(0)
    s = torch.cuda.current_stream()
    ctx.set_stream(s)
    rows = torch.empty(G * k * L, dtype=torch.uint8, device=dev)
    ctx.synth_fixed(rows, k, L, 0, G, 0x51554943)
    miss = torch.from_numpy(np.random.default_rng(1).integers(0, k, G).astype(np.uint8)).to(dev)
    par = torch.empty(G * L, dtype=torch.uint8, device=dev)
    out = torch.empty(G * L, dtype=torch.uint8, device=dev)
    ref = None
    res = {}
    for r in range(rounds):
        for rv in (0, 8, 16):
            ctx.debug_phase_reserve(rv)
            for op in ("enc", "rec"):
                def run():
                    if op == "enc":
                        ctx.encode(rows, k, L, G, par)
                    else:
                        ctx.recover(rows, par, miss, k, L, G, out)
                run()
                grid = ctx.last_phase_grid()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    run()
                e1.record(s)
                e1.synchronize()
                res.setdefault((rv, op), []).append(e0.elapsed_time(e1) / reps / 1e3)
                res[(rv, op, "grid")] = grid
            ctx.sync()
            h = (par.sum().item(), out.sum().item())
            ref = ref or h
            assert h == ref, "outputs differ between grid sizes"
    ctx.debug_phase_reserve(0)
    b = G * (k + 1) * L
    for rv in (0, 8, 16):
        line = {"reserve": rv, "grid": res[(rv, "enc", "grid")]}
        for op in ("enc", "rec"):
            t = float(np.median(res[(rv, op)]))
            line[f"{op}_us"] = round(t * 1e6, 1)
            line[f"{op}_frac"] = round(b / t / 1e9 / HBM, 4)
        print(json.dumps(line), flush=True)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
