"""PCIe probe: H2D alone, D2H alone, and both at once (separate streams),
pinned host buffers, 1 GiB each way, to bound the fused FEC + AEAD leg
(DESIGN §6).  Usage on the GPU box: python tools/pcie_probe.py"""
import json
import time

import torch


def main():
    n = 1 << 30
    h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)
        torch.cuda.synchronize()
        res.setdefault("h2d_GBps", []).append(n / (time.perf_counter() - t) / 1e9)
        t = time.perf_counter()
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
        res.setdefault("d2h_GBps", []).append(n / (time.perf_counter() - t) / 1e9)
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
        res.setdefault("both_total_GBps", []).append(2 * n / (time.perf_counter() - t) / 1e9)
    print(json.dumps({k: round(max(v), 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
