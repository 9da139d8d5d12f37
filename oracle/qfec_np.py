"""NumPy restatement of the QUIC FEC group arithmetic — TEST INFRASTRUCTURE ONLY.

An independent second restatement of SURVEY.md Appendix A, written with
vectorised ``np.bitwise_xor.reduce`` instead of the C oracle's word loop, so
that the two can cross-check each other (tests/test_oracle.py) and so that the
golden fixtures under tests/golden/ are produced by code that shares nothing
with the C oracle or the HIP product path.

PARITY UNPINNED by the reference: the libquic snapshot has no FEC source
(Makefile:5332-5384 names the missing quic_fec_group*.cc;
src/net/quic/core/quic_protocol.h:373) and no FEC vectors.  In-tree constraints
followed: kMaxPacketSize = 1452 (quic_protocol.h:66), k <= 255
(quic_framer.cc:1126-1136), zero padding (quic_data_writer.cc:136-143,
quic_framer.cc:1224-1231), QUIC_INVALID_FEC_DATA = 5 (quic_protocol.h:538).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import it.
"""
from __future__ import annotations

import numpy as np

MAX_PACKET_SIZE = 1452  # kMaxPacketSize, quic_protocol.h:66
MAX_GROUP_PACKETS = 255  # uint8 group offset, quic_framer.cc:1126
INVALID_FEC_DATA = 5  # QUIC_INVALID_FEC_DATA, quic_protocol.h:538

SEED_FIXED = 0x51554943
SEED_RAGGED = 0x51554944
SEED_DROP = 0x51554945

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


class InvalidFecData(ValueError):
    """Raised where the C-ABI returns -QUIC_INVALID_FEC_DATA."""


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_row(seed: int, g: int, i: int, length: int) -> np.ndarray:
    key = np.uint64(seed) ^ (np.uint64(g * 256 + i) << np.uint64(32))
    nw = (length + 7) // 8
    words = splitmix64(key ^ np.arange(nw, dtype=np.uint64))
    return words.astype("<u8").view(np.uint8)[:length].copy()


def synth_fixed(seed: int, g0: int, n: int, k: int, L: int) -> np.ndarray:
    """rows[n, k, L] of the counter-based synthetic input."""
    g = np.arange(g0, g0 + n, dtype=np.uint64)[:, None, None]
    i = np.arange(k, dtype=np.uint64)[None, :, None]
    nw = (L + 7) // 8
    w = np.arange(nw, dtype=np.uint64)[None, None, :]
    key = np.uint64(seed) ^ ((g * np.uint64(256) + i) << np.uint64(32))
    words = splitmix64(key ^ w)
    return words.astype("<u8").view(np.uint8).reshape(n, k, nw * 8)[:, :, :L].copy()


def ragged_k(seed: int, g, kmin: int, kmax: int):
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x6B << 56) ^ np.asarray(g, dtype=np.uint64))
    return (np.uint64(kmin) + h % np.uint64(kmax - kmin + 1)).astype(np.int64)


def ragged_len(seed: int, g, i, lmin: int, lmax: int):
    gi = np.asarray(g, dtype=np.uint64) * np.uint64(256) + np.asarray(i, dtype=np.uint64)
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x4C << 56) ^ gi)
    return (np.uint64(lmin) + h % np.uint64(lmax - lmin + 1)).astype(np.int64)


def drop_index(seed: int, g, k):
    h = splitmix64(np.uint64(seed) ^ np.uint64(0x44 << 56) ^ np.asarray(g, dtype=np.uint64))
    return (h % np.asarray(k, dtype=np.uint64)).astype(np.int64)


def _check_len(n):
    if n < 1 or n > MAX_PACKET_SIZE:
        raise InvalidFecData(f"payload length {n} outside [1, {MAX_PACKET_SIZE}]")


def group_encode(payloads):
    """Parity of one group: XOR of zero-padded payloads; len = max payload len."""
    k = len(payloads)
    if k < 1 or k > MAX_GROUP_PACKETS:
        raise InvalidFecData(f"group size {k}")
    for p in payloads:
        _check_len(len(p))
    plen = max(len(p) for p in payloads)
    pad = np.zeros((k, plen), dtype=np.uint8)
    for r, p in enumerate(payloads):
        pad[r, : len(p)] = np.frombuffer(bytes(p), dtype=np.uint8)
    return np.bitwise_xor.reduce(pad, axis=0)


def group_recover(payloads, parity, m: int):
    """Revive packet m: parity XOR every received payload (zero padded)."""
    k = len(payloads)
    if k < 1 or k > MAX_GROUP_PACKETS or not (0 <= m < k):
        raise InvalidFecData(f"missing index {m} for k={k}")
    parity = np.asarray(parity, dtype=np.uint8)
    _check_len(parity.size)
    acc = parity.copy()
    for r, p in enumerate(payloads):
        if r == m:
            continue
        _check_len(len(p))
        if len(p) > parity.size:
            raise InvalidFecData("payload longer than parity")
        acc[: len(p)] ^= np.frombuffer(bytes(p), dtype=np.uint8)
    return acc


def encode_fixed(rows: np.ndarray) -> np.ndarray:
    """rows[n, k, L] -> parity[n, L]"""
    n, k, L = rows.shape
    if k < 1 or k > MAX_GROUP_PACKETS:
        raise InvalidFecData(f"k={k}")
    _check_len(L)
    return np.bitwise_xor.reduce(rows, axis=1)


def recover_fixed(rows: np.ndarray, parity: np.ndarray, missing: np.ndarray) -> np.ndarray:
    n, k, L = rows.shape
    missing = np.asarray(missing)
    if np.any(missing >= k) or np.any(missing < 0):
        raise InvalidFecData("missing index out of range")
    keep = np.ones((n, k), dtype=bool)
    keep[np.arange(n), missing] = False
    masked = np.where(keep[:, :, None], rows, np.uint8(0))
    return np.bitwise_xor.reduce(masked, axis=1) ^ parity


def ragged_batch(seed: int, g0: int, n: int, kmin=5, kmax=15, lmin=64, lmax=1350,
                 parity_stride=MAX_PACKET_SIZE):
    """Packed CSR ragged batch: (bytes, pkt_off, pkt_len, grp_ptr, parity_off)."""
    gs = np.arange(g0, g0 + n, dtype=np.uint64)
    ks = ragged_k(seed, gs, kmin, kmax)
    grp_ptr = np.zeros(n + 1, dtype=np.uint32)
    grp_ptr[1:] = np.cumsum(ks)
    lens = []
    for gi, k in zip(gs, ks):
        lens.append(ragged_len(seed, int(gi), np.arange(k), lmin, lmax))
    pkt_len = np.concatenate(lens).astype(np.uint16)
    pkt_off = np.zeros(pkt_len.size, dtype=np.uint64)
    pkt_off[1:] = np.cumsum(pkt_len[:-1].astype(np.uint64))
    total = int(pkt_off[-1]) + int(pkt_len[-1])
    data = np.zeros(total, dtype=np.uint8)
    for gidx, gi in enumerate(gs):
        for r in range(int(ks[gidx])):
            p = int(grp_ptr[gidx]) + r
            o, ln = int(pkt_off[p]), int(pkt_len[p])
            data[o : o + ln] = synth_row(seed, int(gi), r, ln)
    parity_off = np.arange(n, dtype=np.uint64) * np.uint64(parity_stride)
    return data, pkt_off, pkt_len, grp_ptr, parity_off


def encode_ragged(data, pkt_off, pkt_len, grp_ptr, parity_off, parity_size):
    n = grp_ptr.size - 1
    parity = np.zeros(parity_size, dtype=np.uint8)
    plen = np.zeros(n, dtype=np.uint16)
    for g in range(n):
        pays = [data[int(pkt_off[p]) : int(pkt_off[p]) + int(pkt_len[p])]
                for p in range(int(grp_ptr[g]), int(grp_ptr[g + 1]))]
        par = group_encode(pays)
        parity[int(parity_off[g]) : int(parity_off[g]) + par.size] = par
        plen[g] = par.size
    return parity, plen


def recover_ragged(data, pkt_off, pkt_len, grp_ptr, parity, parity_off, parity_len,
                   missing, out_off, out_size):
    n = grp_ptr.size - 1
    out = np.zeros(out_size, dtype=np.uint8)
    for g in range(n):
        pays = [data[int(pkt_off[p]) : int(pkt_off[p]) + int(pkt_len[p])]
                for p in range(int(grp_ptr[g]), int(grp_ptr[g + 1]))]
        pl = int(parity_len[g])
        par = parity[int(parity_off[g]) : int(parity_off[g]) + pl]
        rec = group_recover(pays, par, int(missing[g]))
        out[int(out_off[g]) : int(out_off[g]) + pl] = rec
    return out
