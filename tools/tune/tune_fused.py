"""Chunk size / slot count sweep of bench.py's fused FEC + AES-128-GCM-12
host-memory leg (bench_fused), against the measured bidirectional PCIe copy
rate (tools/tune/tune_zero_copy.hip: 97 GB/s total, 48.6 GB/s each way).
Usage: python tools/tune/tune_fused.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from libquic_amd import qfec  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = qfec.Context(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream)
    for cg, slots in ((8192, 3), (4096, 3), (4096, 4), (8192, 4), (16384, 3), (2048, 6),
                      (4096, 6)):
        r = bench.bench_fused(ctx, torch, dev, stream, 10, 1350, cg=cg, slots=slots, cpu=False)
        moved = r["pcie_h2d_bytes"] + r["pcie_d2h_bytes"]
        print(json.dumps({"chunk_groups": cg, "slots": slots, "payload_GiBps": r["payload_GiBps"],
                          "wall_ms": r["wall_ms"], "link_GBps": round(moved / r["wall_ms"] / 1e6, 1),
                          "verified": r["verified"]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
