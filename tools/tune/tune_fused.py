"""Chunking of the fused FEC + AES-128-GCM-12 host-memory leg (bench.bench_fused):
chunk size x slots, payload GiB/s over wall time (pinned host buffers).
python tools/tune/tune_fused.py > gpurun_out/tune_fused.txt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from libquic_amd import qfec  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
ctx = qfec.Context(0)
stream = torch.cuda.current_stream()
ctx.set_stream(stream)
for cg, slots in [(4096, 3), (4096, 4), (8192, 3), (8192, 4), (2048, 4), (2048, 6), (16384, 3)]:
    r = bench.bench_fused(ctx, torch, dev, stream, 10, 1350, cg=cg, slots=slots, cpu=False)
    print(f"cg {cg:6d} slots {slots}: staged {r['payload_GiBps']:6.2f} GiB/s "
          f"({r['wall_ms']:.1f} ms, ok {r['verified']}), direct_out "
          f"{r['direct_out']['payload_GiBps']:6.2f} GiB/s (ok {r['direct_out']['verified']})",
          flush=True)
ctx.close()
