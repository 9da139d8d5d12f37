"""Generate the golden FEC fixtures under tests/golden/ (committed data).

Why generated here: the libquic snapshot has no FEC source and no FEC vectors
(SURVEY.md §0, §8(c) — /root/reference/Makefile:5332-5384 names the removed
quic_fec_group*.cc), so parity is UNPINNED by the reference.  The fixtures are
produced by the NumPy restatement (oracle/qfec_np.py), which shares no code
with the C oracle or the HIP product path, and every fixture is also checked
against the algebraic identities in tests/test_oracle.py.

Files:
  fixed_k10_L1350.npz   8 groups of the headline shape (SURVEY.md §8(d) seeds)
  shapes.npz            edge shapes: k in {1,2,3,255}, L in {1,15,16,17,63,64,1350,1452}
  ragged.npz            24 ragged groups, k 5..15, len 64..1350 (+ a tiny-len group set)
  full_digests.json     checksum-of-checksums of the FULL 1M-group fixed workload,
                        computed by the C oracle (make_golden.py --full)

Run:  python tests/golden/make_golden.py [--full]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import qfec_np as Q  # noqa: E402


def fixed_case(seed, g0, n, k, L):
    rows = Q.synth_fixed(seed, g0, n, k, L)
    parity = Q.encode_fixed(rows)
    missing = Q.drop_index(Q.SEED_DROP, np.arange(g0, g0 + n), k).astype(np.uint8)
    recovered = Q.recover_fixed(rows, parity, missing)
    assert np.array_equal(recovered, rows[np.arange(n), missing])
    return rows, parity, missing, recovered


def main():
    rows, parity, missing, recovered = fixed_case(Q.SEED_FIXED, 0, 8, 10, 1350)
    np.savez_compressed(os.path.join(HERE, "fixed_k10_L1350.npz"), rows=rows, parity=parity,
                        missing=missing, recovered=recovered,
                        meta=np.array([Q.SEED_FIXED, 0, 8, 10, 1350], dtype=np.uint64))

    shapes = {}
    for k, L, n in [(1, 1350, 2), (2, 64, 3), (3, 1, 4), (3, 15, 4), (3, 16, 4), (3, 17, 4),
                    (4, 63, 3), (5, 64, 3), (255, 64, 1), (255, 1452, 1), (10, 1452, 2),
                    (7, 1351, 2)]:
        r, p, m, rec = fixed_case(Q.SEED_FIXED + k * 7 + L, 3, n, k, L)
        tag = f"k{k}_L{L}"
        shapes[f"{tag}_rows"] = r
        shapes[f"{tag}_parity"] = p
        shapes[f"{tag}_missing"] = m
        shapes[f"{tag}_recovered"] = rec
    np.savez_compressed(os.path.join(HERE, "shapes.npz"), **shapes)

    rag = {}
    for tag, (n, kmin, kmax, lmin, lmax) in {"main": (24, 5, 15, 64, 1350),
                                             "tiny": (12, 1, 6, 1, 40)}.items():
        data, off, ln, ptr, poff = Q.ragged_batch(Q.SEED_RAGGED, 5, n, kmin, kmax, lmin, lmax)
        par, plen = Q.encode_ragged(data, off, ln, ptr, poff, n * Q.MAX_PACKET_SIZE)
        ks = np.diff(ptr.astype(np.int64))
        miss = Q.drop_index(Q.SEED_DROP, np.arange(5, 5 + n), ks).astype(np.uint8)
        ooff = np.arange(n, dtype=np.uint64) * np.uint64(Q.MAX_PACKET_SIZE)
        rec = Q.recover_ragged(data, off, ln, ptr, par, poff, plen, miss, ooff,
                               n * Q.MAX_PACKET_SIZE)
        for g in range(n):  # revived == lost packet, zero padded to parity_len
            p = int(ptr[g]) + int(miss[g])
            o, L_ = int(off[p]), int(ln[p])
            seg = rec[int(ooff[g]): int(ooff[g]) + int(plen[g])]
            assert np.array_equal(seg[:L_], data[o:o + L_]) and not seg[L_:].any()
        for name, arr in dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff,
                              parity=par, parity_len=plen, missing=miss, out_off=ooff,
                              recovered=rec).items():
            rag[f"{tag}_{name}"] = arr
    np.savez_compressed(os.path.join(HERE, "ragged.npz"), **rag)

    if "--full" in sys.argv:
        from oracle import oracle_c as OC
        n = 1 << 20
        pd, rd = OC.fixed_digests(Q.SEED_FIXED, Q.SEED_DROP, 0, n, 10, 1350)
        pd2, rd2 = OC.fixed_digests(Q.SEED_FIXED, Q.SEED_DROP, n, n, 10, 1350)
        out = {"seed": Q.SEED_FIXED, "drop_seed": Q.SEED_DROP, "k": 10, "L": 1350,
               "digests": {"g0=0,n=1048576": {"parity": f"{pd:#018x}", "recovered": f"{rd:#018x}"},
                           "g0=1048576,n=1048576": {"parity": f"{pd2:#018x}",
                                                    "recovered": f"{rd2:#018x}"}},
               "definition": "FNV-1a-64 over the little-endian sequence of per-group FNV-1a-64 "
                             "hashes of each group's parity (resp. revived row), group order"}
        with open(os.path.join(HERE, "full_digests.json"), "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
    if "--full" in sys.argv or "--full-ragged" in sys.argv:
        # configs[3] at full size: 2^20 ragged groups, k 5-15,
        # payloads 64-1350 B, parity rows and revived rows (layout independent)
        from oracle import oracle_c as OC
        n = 1 << 20
        path = os.path.join(HERE, "full_digests.json")
        with open(path) as f:
            out = json.load(f)
        pd, rd = OC.ragged_digests(Q.SEED_RAGGED, Q.SEED_DROP, 0, n, 5, 15, 64, 1350)
        out["ragged"] = {"seed": Q.SEED_RAGGED, "drop_seed": Q.SEED_DROP, "k": [5, 15],
                         "len": [64, 1350],
                         "digests": {"g0=0,n=1048576": {"parity": f"{pd:#018x}",
                                                        "recovered": f"{rd:#018x}"}},
                         "definition": "as above, over each group's parity_len bytes of parity "
                                       "(resp. of the revived row: the lost packet zero padded "
                                       "to parity_len); oracle/qfec_oracle.c qo_ragged_digests"}
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
