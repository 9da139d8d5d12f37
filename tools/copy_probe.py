"""Copy ceilings on the box (the roofline the NULL protection kernels sit
under — they are a copy plus a hash): the library's nt 16-B streaming copy
(qfec_stream_probe) and the runtime's device-to-device copy (torch copy_ =
hipMemcpyAsync D2D), 7 GB each way, bytes read + written / time.
Usage on the GPU box: python tools/copy_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libquic_amd import qfec  # noqa: E402


def timed(stream, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 7 << 30
    buf = torch.empty(2 * n, dtype=torch.uint8, device="cuda:0")
    buf.fill_(1)
    ctx = qfec.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s)
    res = {}
    ms = timed(s, lambda: ctx.stream_probe(buf, n, buf[n:], copy=True))
    res["qfec_nt_copy_GBps"] = round(2 * n / ms / 1e6, 1)
    with torch.cuda.stream(s):
        ms = timed(s, lambda: buf[n:].copy_(buf[:n]))
    res["hip_d2d_copy_GBps"] = round(2 * n / ms / 1e6, 1)
    # an unaligned copy (src +2, dst +12: the NULL kernels' packed layout)
    with torch.cuda.stream(s):
        ms = timed(s, lambda: buf[n + 12:2 * n - 4].copy_(buf[2:n - 14]))
    res["hip_d2d_copy_unaligned_GBps"] = round(2 * (n - 16) / ms / 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
