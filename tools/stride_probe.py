"""Fixed-shape FEC batch at several row strides, one process, one set of
buffers (the same placement for every stride): is the headline kernel's rate
a property of its 1350-B packed rows' alignment?

Rows of 1350 B at stride 1350 (packed, configs[1]), 1360 (each payload
rounded to 16 B, as the host payload arena lays payloads out,
quic_fec_group.cc PayloadArena::Alloc), 1408 (11 x 128 B) and 1536.
Algorithmic bytes per launch are the same for every stride (k*L + L per
group); rates are reported against 8 TB/s.  Output rows (parity, revived)
at stride L.  Bench / tuning plumbing only.

usage: python tools/stride_probe.py [groups] [reps] > out.txt
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from libquic_amd import qfec  # noqa: E402
from libquic_amd import synth  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    k, L = 10, 1350
    strides = [1350, 1360, 1408, 1536]
    dev = "cuda:0"
    rows = torch.empty(G * k * max(strides), dtype=torch.uint8, device=dev)
    par = torch.empty(G * L, dtype=torch.uint8, device=dev)
    out = torch.empty(G * L, dtype=torch.uint8, device=dev)
    miss = torch.from_numpy(synth.drop_indices(synth.SEED_DROP, np.arange(G, dtype=np.uint64),
                                               np.full(G, k)).astype(np.uint8)).to(dev)
    alg = G * (k * L + L)
    with qfec.Context(0) as ctx:
        stream = torch.cuda.Stream()
        ctx.set_stream(stream)
        res = {s: ([], []) for s in strides}
        ref = None
        for rnd in range(3):
            for s in strides:
                ctx.synth_fixed(rows, k, L, 0, G, synth.SEED_FIXED, row_stride=s, group_stride=k * s)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ctx.encode(rows, k, L, G, par, row_stride=s, group_stride=k * s)
                ctx.sync()
                ev[0].record(stream)
                for _ in range(reps):
                    ctx.encode(rows, k, L, G, par, row_stride=s, group_stride=k * s)
                ev[1].record(stream)
                for _ in range(reps):
                    ctx.recover(rows, par, miss, k, L, G, out, row_stride=s, group_stride=k * s)
                ev[2].record(stream)
                ctx.sync()
                torch.cuda.synchronize()
                te = ev[0].elapsed_time(ev[1]) / reps / 1e3
                tr = ev[1].elapsed_time(ev[2]) / reps / 1e3
                res[s][0].append(alg / te / 8e12)
                res[s][1].append(alg / tr / 8e12)
                # the same bytes at every stride: parity and revived rows must agree
                h = (par[:1 << 20].cpu().numpy().tobytes(), out[:1 << 20].cpu().numpy().tobytes())
                if ref is None:
                    ref = h
                same = h == ref
                print(f"round {rnd} stride {s}: encode {res[s][0][-1]:.4f} recover "
                      f"{res[s][1][-1]:.4f} of 8 TB/s  outputs equal to stride 1350: {same}",
                      flush=True)
                if not same:
                    raise SystemExit(1)
        print(f"{G} groups x {k} x {L} B, {reps} launches per point; median of 3 rounds:")
        for s in strides:
            e, r = sorted(res[s][0])[1], sorted(res[s][1])[1]
            print(f"stride {s:5d}: encode {e:.4f}  recover {r:.4f}")


if __name__ == "__main__":
    main()
