"""Diagnose ragged recover mismatches on the GPU: which groups differ and how."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_hip_ragged import synth_batch, run_ragged, dview  # noqa: E402
from oracle import oracle_c as OC  # noqa: E402
from oracle import qfec_np as Q  # noqa: E402
from libquic_amd import qfec  # noqa: E402
import torch  # noqa: E402

n = 20_000
ks, ptr, ln, off = synth_batch(n, g0=77)
total = int(off[-1] + ln[-1])
with qfec.Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream())
    data_d = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
    ctx.synth_ragged(data_d, dview(off), dview(ln), dview(ptr), 77, n, Q.SEED_RAGGED)
    ctx.sync()
    data = data_d.cpu().numpy()
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1452)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(77, 77 + n), ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1452)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff, n * 1452)
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z)
    o2 = out.reshape(n, 1452)
    w2 = want_o.reshape(n, 1452)
    bad = np.nonzero((o2 != w2).any(axis=1))[0]
    print("bad groups", bad.size, "of", n)
    for g in bad[:12]:
        p0, p1 = int(ptr[g]), int(ptr[g + 1])
        diff = np.nonzero(o2[g] != w2[g])[0]
        print(f"g={g} k={p1-p0} m={int(miss[g])} plen={want_l[g]} lens={list(ln[p0:p1])} "
              f"lost_len={ln[p0+int(miss[g])]} ndiff={diff.size} first={diff[:8]} last={diff[-4:]}")
    # statistics: is m == argmax(lens)?  plen vs received max
    st = []
    for g in bad:
        p0, p1 = int(ptr[g]), int(ptr[g + 1])
        l = ln[p0:p1].astype(int)
        rec = np.delete(l, int(miss[g]))
        st.append((int(l[int(miss[g])] == l.max()), int(rec.max()), int(want_l[g])))
    st = np.array(st) if st else np.zeros((0, 3))
    if len(st):
        print("lost is the longest:", st[:, 0].mean(), " recvmax<plen:", (st[:, 1] < st[:, 2]).mean())
    allm = [int(ln[int(ptr[g]) + int(miss[g])] == ln[int(ptr[g]):int(ptr[g + 1])].max()) for g in range(n)]
    print("overall lost-is-longest rate", np.mean(allm))
    # dump a few bad groups for offline analysis
    dump = {}
    for j, g in enumerate(bad[:6]):
        p0, p1 = int(ptr[g]), int(ptr[g + 1])
        dump[f"g{j}_out"] = o2[g]
        dump[f"g{j}_want"] = w2[g]
        dump[f"g{j}_par"] = want_p.reshape(n, 1452)[g]
        dump[f"g{j}_lens"] = ln[p0:p1]
        dump[f"g{j}_m"] = np.array([int(miss[g])])
        for i in range(p1 - p0):
            dump[f"g{j}_pkt{i}"] = data[int(off[p0 + i]):int(off[p0 + i]) + int(ln[p0 + i])]
    os.makedirs("gpurun_out/diag", exist_ok=True)
    np.savez("gpurun_out/diag/bad_groups.npz", **dump)
    # repeat the recover: same groups bad again?
    par2, plen2, out2 = run_ragged(ctx, z)
    bad2 = np.nonzero((out2.reshape(n, 1452) != w2).any(axis=1))[0]
    print("second run bad", bad2.size, "overlap", np.intersect1d(bad, bad2).size)
