"""Round 6 measurement: a small-batch service flush end to
end, host and worker, for 1 and 64 groups of 10 x 1350 B in host-mapped
memory (the connection leg's shape).

Each call: qfec_service_warm at the "turn start", a busy wait of `gap` us (the
connection leg's batch assembly between the warm and the flush: 0, 30 or
80 us), then one synchronous QFEC_PTR_MAPPED encode.  The stamps
(qfec_debug_service_trace): the host's steady clock at the call's entry, after
the job is published, when the token is seen and at return; the worker's
100-MHz wall clock when the leader's poll saw the job, when its entry was in
LDS, and for every workgroup when its share's entry was in LDS, its groups
done, its outputs visible, counted; and when the token was stored.  The two
clocks are not compared directly: the host's wait (published -> token seen)
minus the worker's (job seen -> token stored) is the two one-way link
latencies (publish -> poll sees it, token store -> host sees it) together.

  python tools/svc_trace.py [calls=300] [groups=1,64] [gaps=0,30,80]

One JSON line per (groups, gap): medians over the calls (microseconds).
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


def spin_us(us):
    t = time.perf_counter() + us * 1e-6
    while time.perf_counter() < t:
        pass


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    ctx = qfec.Context(0)
    try:
        ctx.debug_service_stamps(True)
        ns = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 64]
        gaps = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 30, 80]
        for n in ns:
            z, _ = _mapped_case(n, g0=5000, kmin=10, kmax=10, lmin=1350, lmax=1350)
            data = qfec.HostBuffer(z["data"].nbytes)
            data.array[:] = z["data"]
            par = qfec.HostBuffer(z["parity"].size)
            plen = np.zeros(n, np.uint16)
            for gap in gaps:
                rows = []
                for it in range(calls):
                    ctx.service_warm()
                    spin_us(gap)
                    ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n,
                                      par.array, z["parity_off"], plen, mapped=True)
                    t = ctx.debug_service_trace()
                    st, wg, h = t[:8], np.array(t[8:40], dtype=np.float64).reshape(8, 4), t[40:44]
                    d = lambda a, b: (a - b) / 100.0  # noqa: E731  (10-ns ticks -> us)
                    active = wg[:, 0] >= st[0] if n > 8 else np.array([True] + [False] * 7)
                    w = wg[active]
                    rows.append({
                        "host_total": (h[3] - h[0]) / 1e3,
                        "host_to_publish": (h[1] - h[0]) / 1e3,
                        "host_wait": (h[2] - h[1]) / 1e3,
                        "host_after_token": (h[3] - h[2]) / 1e3,
                        "worker_seen_to_token": d(st[6] if n > 8 else st[5], st[0]),
                        "leader_entry": d(st[1], st[0]),
                        "entry_last_wg": d(w[:, 0].max(), st[0]),
                        "groups_slowest_wg": float(((w[:, 1] - w[:, 0]) / 100.0).max()),
                        "groups_done_last": d(w[:, 1].max(), st[0]),
                        "fence_max": float(((w[:, 2] - w[:, 1]) / 100.0).max()),
                        "counted_last": d(w[:, 3].max(), st[0]),
                    })
                    rows[-1]["links_two_way"] = rows[-1]["host_wait"] - rows[-1]["worker_seen_to_token"]
                    if n > 8:
                        rows[-1]["token_wg"] = int(st[7])
                assert np.array_equal(par.array, z["parity"]), n
                keep = rows[calls // 4:]
                out = {"groups": n, "gap_us": gap, "calls": len(keep),
                       "launches": ctx.debug_service()["launches"]}
                for key in keep[0]:
                    if key == "token_wg":
                        continue
                    out[key] = round(float(np.median([r[key] for r in keep])), 2)
                print(json.dumps(out), flush=True)
            data.close()
            par.close()
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
