"""The fused FEC + AES-GCM leg (bench.py bench_fused) alone, both copy
schedules (slots / duplex) and the direct-out form, for a few slot counts.
GPU box: python tools/fused_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from libquic_amd import qfec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    ctx = qfec.Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    for slots, cg in ((3, 4096), (3, 16384), (2, 16384), (4, 8192)):
        r = bench.bench_fused(ctx, torch, dev, stream, 10, 1350, cg=cg, slots=slots, cpu=False)
        print(json.dumps({"n_slots": slots, "chunk_groups": cg,
                          **{k: r[k] for k in ("payload_GiBps", "schedule", "duplex", "slots",
                                               "direct_out")}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
