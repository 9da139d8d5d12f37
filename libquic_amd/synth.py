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


def ragged_layout(g0, n, kmin=5, kmax=15, lmin=64, lmax=1350, seed=SEED_RAGGED):
    """Packed CSR layout of n groups: (k, grp_ptr u32, pkt_len u16, pkt_off u64)."""
    gs = np.arange(g0, g0 + n, dtype=np.uint64)
    ks = group_sizes(seed, gs, kmin, kmax)
    ptr = np.zeros(n + 1, np.uint32)
    ptr[1:] = np.cumsum(ks)
    gidx = np.repeat(gs, ks)
    iidx = np.arange(int(ptr[-1]), dtype=np.int64) - np.repeat(ptr[:-1].astype(np.int64), ks)
    ln = packet_lengths(seed, gidx, iidx, lmin, lmax).astype(np.uint16)
    off = np.zeros(ln.size, np.uint64)
    if ln.size > 1:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    return ks, ptr, ln, off
