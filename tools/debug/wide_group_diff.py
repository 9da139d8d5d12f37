"""Round-5 debug: the window_group slot-table rewrite fails on 'wide'
groups (more than 64 slots).  Runs the failing group alone through the
latency kernel (mapped payloads) and names every wrong 16-B parity window
and which packet windows its difference equals."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_hip_mapped import _mapped_case  # noqa: E402
from test_hip_ragged import run_ragged  # noqa: E402

from libquic_amd import qfec  # noqa: E402

z, want_l = _mapped_case(2, g0=1002)
ptr, ln, off, data = z["grp_ptr"], z["pkt_len"], z["pkt_off"], z["data"]
ctx = qfec.Context(0)
par, plen, out = run_ragged(ctx, z, host="mapped")
print("plen", plen, "want", want_l)
g = 1
p0, p1 = int(ptr[g]), int(ptr[g + 1])
po = int(z["parity_off"][g])
L = int(want_l[g])
got = par[po:po + L]
want = z["parity"][po:po + L]
bad = np.nonzero(got != want)[0]
print("group", g, "k", p1 - p0, "plen", L, "wrong bytes", bad.size)
if bad.size:
    wins = sorted(set((bad // 16).tolist()))
    print("wrong 16-B windows (by byte // 16):", wins)
    diff = got ^ want
    for w in wins[:8]:
        lo = w * 16
        d = diff[lo:lo + 16]
        hits = []
        for i in range(p0, p1):
            pk = np.zeros(L, np.uint8)
            n = min(int(ln[i]), L)
            pk[:n] = data[int(off[i]):int(off[i]) + n]
            if np.array_equal(pk[lo:lo + 16], d):
                hits.append(i - p0)
        print(" window", w, "diff", d[:8].tolist(), "equals packet(s)", hits)
    print("packet lens", ln[p0:p1].tolist())
