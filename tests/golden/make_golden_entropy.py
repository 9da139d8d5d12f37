"""Generate tests/golden/entropy.npz from the REFERENCE's own
QuicSentEntropyManager (quic_sent_entropy_manager.cc, compiled from
/root/reference into oracle/_ref/libref_quic.so by oracle/ref/Makefile).
Run in the container that has /root/reference:
    python tests/golden/make_golden_entropy.py

Layout: the qfec_entropy_* batch form (libquic_amd/synth.py entropy_batch) —
entropy, conn_ptr, first_pn, cum_base, ack_conn, largest, claimed, range_ptr,
range_lo, range_hi — plus the reference's answers: ref_cum (GetCumulativeEntropy
of every packet in every window) and ref_ok (IsValidEntropy of every ack).
Edge acks are appended per connection: largest = last recorded + 1, a missing
interval starting below the window, an empty PacketNumberQueue.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from libquic_amd import synth  # noqa: E402
from oracle import ref_quic as R  # noqa: E402


def add_edges(d, rng):
    """Per connection with a non-empty window, three edge acks (appended
    after that connection's acks, keeping largest non-decreasing)."""
    acks = {k: [] for k in ("ack_conn", "largest", "claimed", "ranges")}
    rp = d["range_ptr"]
    per = {}
    for q, c in enumerate(d["ack_conn"]):
        per.setdefault(int(c), []).append(q)
    out = {k: [] for k in ("ack_conn", "largest", "claimed")}
    lo, hi, ptr = [], [], [0]
    for c in range(d["conn_ptr"].size - 1):
        for q in per.get(c, []):
            out["ack_conn"].append(c)
            out["largest"].append(int(d["largest"][q]))
            out["claimed"].append(int(d["claimed"][q]))
            lo += list(d["range_lo"][rp[q]:rp[q + 1]])
            hi += list(d["range_hi"][rp[q]:rp[q + 1]])
            ptr.append(len(lo))
        f = int(d["first_pn"][c])
        n = len(d["full"][c])
        if n < f:
            continue
        e = d["full"][c]
        # empty queue, largest = last: the true hash
        out["ack_conn"].append(c); out["largest"].append(n)
        out["claimed"].append(int(np.bitwise_xor.reduce(e[:n]))); ptr.append(len(lo))
        # a missing interval starting below the window (f > 1 only)
        if f > 1:
            out["ack_conn"].append(c); out["largest"].append(n)
            out["claimed"].append(int(rng.integers(0, 256)))
            lo.append(f - 1); hi.append(min(f + 1, n + 1)); ptr.append(len(lo))
        # largest beyond the largest recorded packet
        out["ack_conn"].append(c); out["largest"].append(n + 1)
        out["claimed"].append(int(np.bitwise_xor.reduce(e[:n]))); ptr.append(len(lo))
    d["ack_conn"] = np.array(out["ack_conn"], np.uint32)
    d["largest"] = np.array(out["largest"], np.uint64)
    d["claimed"] = np.array(out["claimed"], np.uint8)
    d["range_ptr"] = np.array(ptr, np.uint32)
    d["range_lo"] = np.array(lo, np.uint64)
    d["range_hi"] = np.array(hi, np.uint64)


def reference_answers(d):
    n_conns = d["conn_ptr"].size - 1
    ref_cum = np.zeros(d["entropy"].size, np.uint8)
    ref_ok = np.zeros(d["ack_conn"].size, np.uint8)
    rp = d["range_ptr"]
    for c in range(n_conns):
        sel = np.nonzero(d["ack_conn"] == c)[0]
        counts = [int(rp[q + 1] - rp[q]) for q in sel]
        ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
        lo = np.concatenate([d["range_lo"][rp[q]:rp[q + 1]] for q in sel] + [np.zeros(0, np.uint64)])
        hi = np.concatenate([d["range_hi"][rp[q]:rp[q + 1]] for q in sel] + [np.zeros(0, np.uint64)])
        cum, ok = R.sent_entropy_run(d["full"][c], int(d["first_pn"][c]),
                                     d["largest"][sel].astype(np.uint64), d["claimed"][sel],
                                     ptr, lo.astype(np.uint64), hi.astype(np.uint64))
        b, e = int(d["conn_ptr"][c]), int(d["conn_ptr"][c + 1])
        ref_cum[b:e] = cum
        ref_ok[sel] = ok
    return ref_cum, ref_ok


def main():
    assert R.build(), "reference build failed (needs /root/reference)"
    rng = np.random.default_rng(0x454E54)
    d = synth.entropy_batch(rng, 160, max_packets=400)
    add_edges(d, rng)
    ref_cum, ref_ok = reference_answers(d)
    full = d.pop("full")
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "entropy.npz"),
                        ref_cum=ref_cum, ref_ok=ref_ok, **d)
    print(f"{d['conn_ptr'].size - 1} connections, {d['entropy'].size} packets, "
          f"{d['ack_conn'].size} acks ({int(ref_ok.sum())} valid)")
    del full


if __name__ == "__main__":
    main()
