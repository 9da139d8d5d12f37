"""Round 5 measurement: where a small-batch service job's time goes.

For 1, 8, 16, 32 and 64 groups of 10 x 1350 B (payloads in host-mapped
memory, the connection leg's shape) the worker's wall-clock stamps of the last
job (qfec_debug_service_stamps: work seen, entry in LDS, wave 0's first group,
every group, fence, token) beside the host's time per encode call.  Prints one
JSON line per batch size (medians over the calls, microseconds).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from libquic_amd import qfec  # noqa: E402
from test_hip_mapped import _mapped_case  # noqa: E402

CALLS = int(os.environ.get("SVC_CALLS", "300"))


def main():
    ctx = qfec.Context(0)
    try:
        ctx.debug_service_stamps(True)
        for n in (1, 8, 16, 32, 64):
            z, _ = _mapped_case(n, g0=5000, kmin=10, kmax=10, lmin=1350, lmax=1350)
            data = qfec.HostBuffer(z["data"].nbytes)
            data.array[:] = z["data"]
            par = qfec.HostBuffer(z["parity"].size)
            plen = np.zeros(n, np.uint16)
            host, seg = [], []
            for it in range(CALLS):
                t0 = time.perf_counter()
                ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n,
                                  par.array, z["parity_off"], plen, mapped=True)
                host.append((time.perf_counter() - t0) * 1e6)
                st = ctx.debug_service_stamps()
                seg.append([(st[q + 1] - st[q]) / 100.0 for q in range(5)])
            assert np.array_equal(par.array, z["parity"]), n
            s = np.median(np.array(seg[CALLS // 4:]), axis=0)
            print(json.dumps({"groups": n, "host_us": round(float(np.median(host[CALLS // 4:])), 2),
                              "entry_us": round(float(s[0]), 2),
                              "first_group_us": round(float(s[1]), 2),
                              "rest_groups_us": round(float(s[2]), 2),
                              "fence_us": round(float(s[3]), 2),
                              "token_us": round(float(s[4]), 2),
                              "launches": ctx.debug_service()["launches"]}), flush=True)
            data.close()
            par.close()
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
