"""Synthetic workload shapes — bench/test plumbing.

Counter-based generators so host and device agree without transfers:
  k_g   = kmin + splitmix64(seed ^ 0x6B<<56 ^ g) % (kmax-kmin+1)
  len   = lmin + splitmix64(seed ^ 0x4C<<56 ^ (g*256+i)) % (lmax-lmin+1)
  m_g   = splitmix64(seed ^ 0x44<<56 ^ g) % k_g           (lost packet index)
Packet bytes themselves are generated on the device (qfec_synth_fixed /
qfec_synth_ragged).  No FEC arithmetic here.
"""
from __future__ import annotations

import numpy as np

SEED_FIXED = 0x51554943
SEED_RAGGED = 0x51554944
SEED_DROP = 0x51554945


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def group_sizes(seed, g, kmin, kmax):
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x6B << 56) ^ np.asarray(g, dtype=np.uint64))
    return (np.uint64(kmin) + h % np.uint64(kmax - kmin + 1)).astype(np.int64)


def packet_lengths(seed, g, i, lmin, lmax):
    gi = np.asarray(g, dtype=np.uint64) * np.uint64(256) + np.asarray(i, dtype=np.uint64)
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x4C << 56) ^ gi)
    return (np.uint64(lmin) + h % np.uint64(lmax - lmin + 1)).astype(np.int64)


def drop_indices(seed, g, k):
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x44 << 56) ^ np.asarray(g, dtype=np.uint64))
    return (h % np.asarray(k, dtype=np.uint64)).astype(np.int64)


def ragged_layout(g0, n, kmin=5, kmax=15, lmin=64, lmax=1350, seed=SEED_RAGGED, align=1):
    """CSR layout of n groups: (k, grp_ptr u32, pkt_len u16, pkt_off u64).

    align=1: byte-packed payloads.  align=16: each payload starts on a 16-B
    boundary (≤ 15 B of gap after each), which is the layout the host side's
    payload arena hands the kernels (quic_fec_group.cc PayloadArena::Alloc)."""
    gs = np.arange(g0, g0 + n, dtype=np.uint64)
    ks = group_sizes(seed, gs, kmin, kmax)
    ptr = np.zeros(n + 1, np.uint32)
    ptr[1:] = np.cumsum(ks)
    gidx = np.repeat(gs, ks)
    iidx = np.arange(int(ptr[-1]), dtype=np.int64) - np.repeat(ptr[:-1].astype(np.int64), ks)
    ln = packet_lengths(seed, gidx, iidx, lmin, lmax).astype(np.uint16)
    off = np.zeros(ln.size, np.uint64)
    if ln.size > 1:
        step = ln[:-1].astype(np.uint64)
        if align > 1:
            a = np.uint64(align)
            step = (step + a - np.uint64(1)) // a * a
        off[1:] = np.cumsum(step)
    return ks, ptr, ln, off


def entropy_batch(rng, n_conns, max_packets=300, acks_per_conn=3, max_ranges=4,
                  corrupt=0.3):
    """Synthetic entropy workload (host numpy), ragged: connection c sent
    packets 1..N_c with random entropy bits (hash = flag << (pn % 8),
    quic_framer.cc:351-354), its window starts at first_pn[c] (packets before it
    cleared, their XOR carried in cum_base[c]); each connection gets acks with
    non-decreasing largest_observed, disjoint missing intervals inside the
    window, and a claimed hash that is the true one (what a peer that received
    the acknowledged packets sends) or, with probability `corrupt`, a wrong one.
    Returns a dict of arrays in the qfec_entropy_* layout plus `full` (the
    per-connection hashes of packets 1..N_c, for the reference)."""
    full, first, windows = [], [], []
    for _ in range(n_conns):
        n = int(rng.integers(0, max_packets + 1))
        pn = np.arange(1, n + 1, dtype=np.uint64)
        flags = rng.integers(0, 2, n).astype(np.uint8)
        e = (flags << (pn % np.uint64(8)).astype(np.uint8)).astype(np.uint8)
        f = int(rng.integers(1, n + 2))
        full.append(e)
        first.append(f)
        windows.append(e[f - 1:])
    conn_ptr = np.zeros(n_conns + 1, np.uint64)
    conn_ptr[1:] = np.cumsum([w.size for w in windows])
    entropy = np.concatenate(windows) if n_conns else np.zeros(0, np.uint8)
    cum_base = np.array([np.bitwise_xor.reduce(e[:f - 1]) if f > 1 else 0
                         for e, f in zip(full, first)], np.uint8)
    ack_conn, largest, claimed, rptr, lo, hi = [], [], [], [0], [], []
    for c, (e, f) in enumerate(zip(full, first)):
        n = e.size
        if n < f:
            continue
        ls = np.sort(rng.integers(f, n + 1, acks_per_conn))
        for L in ls:
            L = int(L)
            # disjoint intervals in [f, L]
            cuts = np.sort(rng.choice(np.arange(f, L + 2), size=min(2 * int(rng.integers(0, max_ranges + 1)), L + 2 - f), replace=False)) if L + 2 - f > 0 else []
            h = int(np.bitwise_xor.reduce(e[:L])) if L else 0
            for i in range(0, len(cuts) - 1, 2):
                a, b = int(cuts[i]), int(cuts[i + 1])
                if a < b:
                    lo.append(a)
                    hi.append(b)
                    h ^= int(np.bitwise_xor.reduce(e[a - 1:b - 1]))
            rptr.append(len(lo))
            if rng.random() < corrupt:
                h ^= int(rng.integers(1, 256))
            ack_conn.append(c)
            largest.append(L)
            claimed.append(h)
    return {"entropy": entropy, "conn_ptr": conn_ptr, "first_pn": np.array(first, np.uint64),
            "cum_base": cum_base, "ack_conn": np.array(ack_conn, np.uint32),
            "largest": np.array(largest, np.uint64), "claimed": np.array(claimed, np.uint8),
            "range_ptr": np.array(rptr, np.uint32), "range_lo": np.array(lo, np.uint64),
            "range_hi": np.array(hi, np.uint64), "full": full}


def synth_fixed_host(seed, g0, n, k, L):
    """rows[n*k*L] of the counter-based generator on the host (the formula of
    the device's qfec_synth_fixed: word w of row (g, i) = splitmix64(seed ^
    (g*256 + i) << 32 ^ w), little-endian).  Plumbing for bench.py's CPU
    stand-in workload (multi-rank tests without a GPU); small n only."""
    g = np.arange(g0, g0 + n, dtype=np.uint64)[:, None, None]
    i = np.arange(k, dtype=np.uint64)[None, :, None]
    nw = (L + 7) // 8
    w = np.arange(nw, dtype=np.uint64)[None, None, :]
    with np.errstate(over="ignore"):
        key = np.uint64(seed) ^ ((g * np.uint64(256) + i) << np.uint64(32))
    words = splitmix64(key ^ w)
    return np.ascontiguousarray(
        words.astype("<u8").view(np.uint8).reshape(n, k, nw * 8)[:, :, :L]).reshape(-1)
