"""GPU parity tests of the ragged (CSR) HIP path and of the C++ QuicFecGroup
host mirror, through the C-ABI, against the golden fixtures and the oracle."""
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import oracle_c as OC
from oracle import qfec_np as Q
from libquic_amd import qfec

from conftest import ROOT

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).ravel().copy()).to(DEV)


_SIGNED = {np.dtype(np.uint8): np.uint8, np.dtype(np.uint16): np.int16,
           np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}


def dview(a):
    """device copy of an index array (bits preserved; torch lacks wide unsigned types)"""
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(_SIGNED[a.dtype]).copy()).to(DEV)


def run_ragged(ctx, z, host=False, small=False):
    """host: False = device pointers, True = QFEC_PTR_HOST (staged), "mapped" =
    QFEC_PTR_MAPPED (payloads in qfec_host_alloc memory, read in place);
    small: the QFEC_SMALL_GROUPS hint (device pointers: two groups per wave)."""
    n = z["grp_ptr"].size - 1
    psize = z["parity"].size
    if host == "mapped":
        data = qfec.HostBuffer(max(1, z["data"].nbytes))
        data.array[:z["data"].nbytes] = z["data"].view(np.uint8).ravel()
        par = qfec.HostBuffer(psize)
        par.array[:] = 0
        plen = np.zeros(n, np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                          z["parity_off"], plen, mapped=True)
        out = qfec.HostBuffer(z["recovered"].size)
        out.array[:] = 0
        ctx.recover_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                           z["parity_off"], plen, z["missing"], out.array, z["out_off"],
                           mapped=True)
        return par.array.copy(), plen, out.array.copy()
    if host:
        par = np.zeros(psize, np.uint8)
        plen = np.zeros(n, np.uint16)
        ctx.encode_ragged(z["data"], z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par,
                          z["parity_off"], plen, host=True)
        out = np.zeros(z["recovered"].size, np.uint8)
        ctx.recover_ragged(z["data"], z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par,
                           z["parity_off"], plen, z["missing"], out, z["out_off"], host=True)
        return par, plen, out
    d = {k: dview(v) for k, v in z.items() if k in ("pkt_off", "pkt_len", "grp_ptr", "parity_off",
                                                   "missing", "out_off")}
    data = dev(z["data"])
    par = torch.zeros(psize, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(n, dtype=torch.int16, device=DEV)
    ctx.encode_ragged(data, d["pkt_off"], d["pkt_len"], d["grp_ptr"], n, par, d["parity_off"],
                      plen, small_groups=small)
    out = torch.zeros(z["recovered"].size, dtype=torch.uint8, device=DEV)
    ctx.recover_ragged(data, d["pkt_off"], d["pkt_len"], d["grp_ptr"], n, par, d["parity_off"],
                       plen, d["missing"], out, d["out_off"], small_groups=small)
    ctx.sync()
    torch.cuda.synchronize()
    return par.cpu().numpy(), plen.cpu().numpy().view(np.uint16), out.cpu().numpy()


def sub(golden, tag):
    return {k[len(tag) + 1:]: v for k, v in golden.items() if k.startswith(tag + "_")}


@pytest.mark.parametrize("tag", ["main", "tiny"])
@pytest.mark.parametrize("host", [False, True, "mapped"])
def test_golden_ragged(ctx, golden_ragged, tag, host):
    z = sub(golden_ragged, tag)
    par, plen, out = run_ragged(ctx, z, host=host)
    assert np.array_equal(plen, z["parity_len"])
    assert np.array_equal(par, z["parity"])
    assert np.array_equal(out, z["recovered"])


def synth_batch(n, kmin=5, kmax=15, lmin=64, lmax=1350, g0=0, seed=Q.SEED_RAGGED, align=1):
    """CSR shapes from the seeded generators; bytes filled on the host by the oracle.
    align=16: payloads on 16-B boundaries (the host payload arena's layout)."""
    gs = np.arange(g0, g0 + n, dtype=np.uint64)
    ks = Q.ragged_k(seed, gs, kmin, kmax)
    ptr = np.zeros(n + 1, np.uint32)
    ptr[1:] = np.cumsum(ks)
    gidx = np.repeat(gs, ks)
    iidx = np.arange(ptr[-1]) - np.repeat(ptr[:-1].astype(np.int64), ks)
    ln = Q.ragged_len(seed, gidx, iidx, lmin, lmax).astype(np.uint16)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum((ln[:-1].astype(np.uint64) + np.uint64(align - 1))
                        // np.uint64(align) * np.uint64(align))
    return ks, ptr, ln, off


@pytest.mark.parametrize("align,slot", [(1, 1452), (16, 1536)])
def test_ragged_synth_vs_oracle(ctx, align, slot):
    """Whole-batch parity: byte-packed payloads with kMaxPacketSize parity
    slots, and bench.py's default line (16-B-aligned payloads, 1,536-B slots)."""
    n = 20_000
    ks, ptr, ln, off = synth_batch(n, g0=77, align=align)
    total = int(off[-1] + ln[-1])
    # gaps between aligned payloads hold 0xA5: a last window loaded in place
    # (ragged_block_kernel AL) must mask them, not rely on zeros
    data_d = torch.full((total,), 0xA5, dtype=torch.uint8, device=DEV)
    ctx.synth_ragged(data_d, dview(off), dview(ln), dview(ptr), 77, n, Q.SEED_RAGGED)
    ctx.sync()
    data = data_d.cpu().numpy()
    # device bytes == oracle bytes for a sample of packets
    for p in np.random.default_rng(0).choice(ln.size, 200, replace=False):
        g = int(np.searchsorted(ptr, p, side="right") - 1)
        i = int(p - ptr[g])
        want = np.zeros(int(ln[p]), np.uint8)
        OC.lib().qo_synth_row(Q.SEED_RAGGED, 77 + g, i, int(ln[p]), OC._p(want))
        assert np.array_equal(data[int(off[p]):int(off[p]) + int(ln[p])], want)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(slot)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(77, 77 + n), ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * slot)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * slot)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z)
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


def test_ragged_edges(ctx):
    # k = 1, k = 255, len 1..1452, len < 16 mixed with long packets, scattered offsets
    rng = np.random.default_rng(3)
    groups = [[1452], [1], [15, 1452, 16, 17], [3] * 255, list(rng.integers(1, 1453, 255)),
              [64, 1350], [16], [17, 1]]
    ln = np.array([l for g in groups for l in g], np.uint16)
    ptr = np.zeros(len(groups) + 1, np.uint32)
    ptr[1:] = np.cumsum([len(g) for g in groups])
    gap = rng.integers(0, 40, ln.size).astype(np.uint64)  # unaligned, gapped offsets
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gap[:-1])
    data = rng.integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    n = len(groups)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1500) + np.uint64(3)
    miss = np.array([rng.integers(0, len(g)) for g in groups], np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1500 + 3)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1500 + 3)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    for host in (False, True, "mapped"):
        par, plen, out = run_ragged(ctx, z, host=host)
        assert np.array_equal(plen, want_l)
        assert np.array_equal(par, want_p)
        assert np.array_equal(out, want_o)


def test_ragged_errors(ctx):
    def call(ln, ptr, miss=None, plen=None):
        n = ptr.size - 1
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        data = np.zeros(max(int(ln.astype(np.int64).sum()), 1), np.uint8)
        poff = np.arange(n, dtype=np.uint64) * np.uint64(1452)
        if miss is None:
            ctx.encode_ragged(dev(data), dview(off), dview(ln), dview(ptr), n,
                              torch.zeros(n * 1452, dtype=torch.uint8, device=DEV),
                              dview(poff), torch.zeros(n, dtype=torch.int16, device=DEV))
        else:
            ctx.recover_ragged(dev(data), dview(off), dview(ln), dview(ptr), n,
                               torch.zeros(n * 1452, dtype=torch.uint8, device=DEV),
                               dview(poff), dview(plen), dview(miss),
                               torch.zeros(n * 1452, dtype=torch.uint8, device=DEV), dview(poff))
        ctx.sync()

    with pytest.raises(qfec.InvalidFecData):
        call(np.array([1453], np.uint16), np.array([0, 1], np.uint32))      # > kMaxPacketSize
    with pytest.raises(qfec.InvalidFecData):
        call(np.array([0, 5], np.uint16), np.array([0, 2], np.uint32))      # empty payload
    with pytest.raises(qfec.InvalidFecData):
        call(np.array([5], np.uint16), np.array([0, 1, 1], np.uint32))      # group of 0 packets
    with pytest.raises(qfec.InvalidFecData):
        call(np.array([5] * 256, np.uint16), np.array([0, 256], np.uint32))  # 256 packets
    with pytest.raises(qfec.InvalidFecData):  # missing index >= k
        call(np.array([5, 5], np.uint16), np.array([0, 2], np.uint32), np.array([2], np.uint8),
             np.array([5], np.uint16))
    with pytest.raises(qfec.InvalidFecData):  # received packet longer than the redundancy
        call(np.array([5, 9], np.uint16), np.array([0, 2], np.uint32), np.array([0], np.uint8),
             np.array([5], np.uint16))
    with pytest.raises(qfec.InvalidFecData):  # redundancy length 0
        call(np.array([5, 5], np.uint16), np.array([0, 2], np.uint32), np.array([0], np.uint8),
             np.array([0], np.uint16))
    # valid call after errors works
    call(np.array([5, 5], np.uint16), np.array([0, 2], np.uint32))


def test_cpp_quic_fec_group():
    """C++ host mirror (QuicFecGroup + wire format) against the oracle."""
    exe = os.path.join(ROOT, "tests", "cpp", "build", "test_quic_fec_group")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert " 0 failures" in r.stdout


@pytest.mark.parametrize("host,small", [(False, False), (False, True), (True, False),
                                        ("mapped", False)])
def test_ragged_pair_boundaries(ctx, host, small):
    """ragged_multi_kernel (round 2's product; since round 6 the kernel of
    batches of small groups: QFEC_SMALL_GROUPS, small=True) runs two
    consecutive groups per wave in one flat window space when their received
    packets fit the 64-lane table, all are >= 16 B and every field is valid;
    otherwise the per-group body.  Its switch points (for the block kernel,
    small=False, a shape test: these 17 groups are blocks of 8 with mixed
    fits and fallbacks).
    Pairs straddling each switch: 63 / 64 / 65 received packets (encode: k;
    recover: k - 1), a packet below 16 B in one group, a redundancy shorter
    than 16 B, k = 1 next to k = 255, and an odd group count (the last wave
    holds one group).  Against the oracle, bit-exact."""
    rng = np.random.default_rng(11)

    def grp(k, lo=16, hi=1452):
        return list(rng.integers(lo, hi + 1, k))
    groups = [grp(32), grp(31),          # 63 received (encode), 61 (recover)
              grp(32), grp(32),          # 64 / 62
              grp(32), grp(33),          # 65 / 63
              grp(33), grp(33),          # 66 / 64: recover fits, encode falls back
              grp(33), grp(34),          # 67 / 65
              grp(5) + [15], grp(6),     # a packet below 16 B: both fall back
              [10, 12], grp(3),          # redundancy below 16 B (recover fallback)
              grp(1), grp(255, 1, 1452),  # k = 1 next to k = 255
              grp(7)]                    # odd count: one group in the last wave
    ln = np.array([l for g in groups for l in g], np.uint16)
    ptr = np.zeros(len(groups) + 1, np.uint32)
    ptr[1:] = np.cumsum([len(g) for g in groups])
    gap = rng.integers(0, 9, ln.size).astype(np.uint64)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gap[:-1])
    data = rng.integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    n = len(groups)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1460) + np.uint64(5)
    miss = np.array([rng.integers(0, len(g)) for g in groups], np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1460 + 5)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1460 + 5)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z, host=host, small=small)
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


@pytest.mark.parametrize("host,small", [(False, True), (False, False), (True, False),
                                        ("mapped", False)])
@pytest.mark.parametrize("shape", ["k2-4", "short"])
def test_ragged_small_groups(ctx, host, small, shape):
    """Round 6's shape-aware choice: a large batch whose groups carry few
    bytes (k 2-4 of 16-1452 B, or k 5-15 of 16-400 B: under 4 KiB a group on
    average) runs two groups per wave -- on device pointers with the
    QFEC_SMALL_GROUPS hint, on host / mapped tables by the host's own count
    (those batches here exceed the small-batch paths: 3,001 groups).  The
    same batch without the hint runs the block kernel.  Bit-exact against the
    oracle either way."""
    rng = np.random.default_rng(31 if shape == "k2-4" else 32)
    n = 3001
    ks = rng.integers(2, 5, n) if shape == "k2-4" else rng.integers(5, 16, n)
    hi = 1452 if shape == "k2-4" else 400
    ln = rng.integers(16, hi + 1, int(ks.sum())).astype(np.uint16)
    ptr = np.zeros(n + 1, np.uint32)
    ptr[1:] = np.cumsum(ks)
    assert ln.astype(np.int64).sum() < 4096 * n  # the small-group side of the rule
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(((ln[:-1].astype(np.uint64) + 15) // 16) * 16)
    data = rng.integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1456)
    miss = (rng.integers(0, 1 << 30, n) % ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1456)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1456)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z, host=host, small=small)
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


@pytest.mark.parametrize("host", [False, True, "mapped"])
def test_ragged_block_boundaries(ctx, host):
    """launch_ragged runs eight consecutive groups per 4-wave block in one
    flat window space (ragged_block_kernel) when their received packets fit
    the 256-lane packet table, their windows fit the 16,384-window start
    mask, every packet is >= 16 B and every field is valid; otherwise the
    per-group body.  Blocks straddling each switch: 256 / 257 received
    packets (encode) and 248 / 249 / 256 (recover), 16,016 windows (fits) and
    16,744 (falls back), k = 1 groups on the fast path (recover: no received
    packet, the revived packet is the redundancy), a packet below 16 B, and a
    partial last block.  Against the oracle, bit-exact."""
    rng = np.random.default_rng(12)

    def grp(k, lo=16, hi=1452):
        return list(rng.integers(lo, hi + 1, k))
    groups = ([grp(32) for _ in range(8)]                       # 256 / 248
              + [grp(32) for _ in range(7)] + [grp(33)]        # 257 / 249
              + [grp(33) for _ in range(8)]                    # 264 / 256
              + [grp(22, 1452) for _ in range(8)]              # 16,016 windows
              + [grp(23, 1452) for _ in range(8)]              # 16,744 / 16,016
              + [grp(1), grp(1), grp(1), grp(1), grp(5), [16], grp(2), grp(3)]
              + [grp(5) + [15], grp(6), grp(4), grp(9), grp(3), grp(2), grp(7), grp(1)]
              + [grp(4), grp(11), grp(1)])                     # partial last block
    ln = np.array([l for g in groups for l in g], np.uint16)
    ptr = np.zeros(len(groups) + 1, np.uint32)
    ptr[1:] = np.cumsum([len(g) for g in groups])
    gap = rng.integers(0, 9, ln.size).astype(np.uint64)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gap[:-1])
    data = rng.integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    n = len(groups)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1460) + np.uint64(5)
    miss = np.array([rng.integers(0, len(g)) for g in groups], np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1460 + 5)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1460 + 5)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z, host=host)
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


def test_ragged_large_batch_odd_groups(ctx):
    """A large device batch (~213K groups) with odd groups mixed in (65-200
    received packets: a block of 8 groups then holds up to ~270, some blocks
    over the 256-lane packet table and some under it; packets < 16 B take the
    per-group body of ragged_block_kernel): parity, lengths and revived
    packets against the
    oracle on sampled groups, the odd ones among them."""
    n = 212_992 + 333
    gs = np.arange(n, dtype=np.uint64)
    ks = Q.ragged_k(Q.SEED_RAGGED, gs, 5, 15)
    rng = np.random.default_rng(11)
    big = rng.choice(n, 40, replace=False)
    ks[big] = rng.integers(65, 200, big.size)  # > 64 received packets
    ptr = np.zeros(n + 1, np.uint32)
    ptr[1:] = np.cumsum(ks)
    gidx = np.repeat(gs, ks)
    iidx = np.arange(ptr[-1]) - np.repeat(ptr[:-1].astype(np.int64), ks)
    ln = Q.ragged_len(Q.SEED_RAGGED, gidx, iidx, 64, 1350).astype(np.uint16)
    short = rng.choice(ln.size, 300, replace=False)
    ln[short] = rng.integers(1, 16, short.size)  # packets below 16 B
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    total = int(off[-1] + ln[-1])
    data = torch.empty(total, dtype=torch.uint8, device=DEV)
    d_off, d_ln, d_ptr = dview(off), dview(ln), dview(ptr)
    ctx.synth_ragged(data, d_off, d_ln, d_ptr, 0, n, Q.SEED_RAGGED)
    miss = Q.drop_index(Q.SEED_DROP, gs, ks).astype(np.uint8)
    poff = gs * np.uint64(1460) + np.uint64(5)
    d_poff, d_miss = dview(poff), dview(miss)
    size = n * 1460 + 5
    pp = torch.full((size,), 0xA5, dtype=torch.uint8, device=DEV)
    pl = torch.zeros(n, dtype=torch.int16, device=DEV)
    ctx.encode_ragged(data, d_off, d_ln, d_ptr, n, pp, d_poff, pl)
    po = torch.full((size,), 0x5A, dtype=torch.uint8, device=DEV)
    ctx.recover_ragged(data, d_off, d_ln, d_ptr, n, pp, d_poff, pl, d_miss, po, d_poff)
    ctx.sync()
    torch.cuda.synchronize()
    # oracle on sampled groups (the big and short ones among them)
    data_h = data.cpu().numpy()
    par_h, plen_h, out_h = pp.cpu().numpy(), pl.cpu().numpy().view(np.uint16), po.cpu().numpy()
    pg = np.searchsorted(ptr, short, side="right") - 1
    sample = np.unique(np.concatenate([big[:10], pg[:20], rng.choice(n, 40, replace=False),
                                       [0, n - 1]]))
    for g in sample:
        g = int(g)
        a, b = int(ptr[g]), int(ptr[g + 1])
        sub_ln = ln[a:b].copy()
        sub_data = np.concatenate([data_h[int(off[q]):int(off[q]) + int(ln[q])] for q in range(a, b)])
        sub_off = np.zeros(b - a, np.uint64)
        sub_off[1:] = np.cumsum(sub_ln[:-1].astype(np.uint64))
        sub_ptr = np.array([0, b - a], np.uint32)
        zp = np.zeros(1, np.uint64)
        rc, wp, wl = OC.encode_ragged(sub_data, sub_off, sub_ln, sub_ptr, zp, 1460)
        rc2, wo = OC.recover_ragged(sub_data, sub_off, sub_ln, sub_ptr, wp, zp, wl,
                                    miss[g:g + 1], zp, 1460)
        assert rc == 0 and rc2 == 0
        L = int(wl[0])
        assert int(plen_h[g]) == L, g
        o = int(poff[g])
        assert np.array_equal(par_h[o:o + L], wp[:L]), g
        assert np.array_equal(out_h[o:o + L], wo[:L]), g


@pytest.mark.parametrize("align,slot", [(16, 1536), (1, 1452)])
def test_full_size_ragged_digest(ctx, align, slot):
    """configs[3] at full size: 2^20 groups, k 5-15,
    payloads 64-1350 B, on the bench's layouts (16-B-aligned payloads with
    1,536-B slots, and byte-packed with 1,452-B slots): the parity rows and
    the revived rows against the committed oracle digests
    (tests/golden/full_digests.json "ragged", oracle qo_ragged_digests), and
    every group's revived row equal to its lost packet on the device."""
    import json
    import os
    from conftest import GOLDEN
    from libquic_amd import synth
    with open(os.path.join(GOLDEN, "full_digests.json")) as f:
        dg = json.load(f)["ragged"]["digests"]["g0=0,n=1048576"]
    G = 1 << 20
    ks, ptr, ln, off = synth.ragged_layout(0, G, 5, 15, 64, 1350, Q.SEED_RAGGED, align=align)
    miss = synth.drop_indices(Q.SEED_DROP, np.arange(G, dtype=np.uint64), ks).astype(np.uint8)
    poff = np.arange(G, dtype=np.uint64) * np.uint64(slot)
    data = torch.full((int(off[-1]) + int(ln[-1]),), 0x77, dtype=torch.uint8, device=DEV)
    t_off, t_len, t_ptr = dview(off), dview(ln), dview(ptr)
    t_poff = dview(poff)
    ctx.synth_ragged(data, t_off, t_len, t_ptr, 0, G, Q.SEED_RAGGED)
    par = torch.full((G * slot,), 0xA5, dtype=torch.uint8, device=DEV)
    plen = torch.zeros(G, dtype=torch.int16, device=DEV)
    out = torch.full((G * slot,), 0x5A, dtype=torch.uint8, device=DEV)
    ctx.encode_ragged(data, t_off, t_len, t_ptr, G, par, t_poff, plen)
    ctx.recover_ragged(data, t_off, t_len, t_ptr, G, par, t_poff, plen, dview(miss), out, t_poff)
    ctx.sync()
    torch.cuda.synchronize()
    plen_h = plen.cpu().numpy().view(np.uint16)
    assert np.array_equal(plen_h, np.maximum.reduceat(ln, ptr[:-1].astype(np.int64)))
    par_h, out_h = par.cpu().numpy(), out.cpu().numpy()
    assert f"{OC.group_digest(par_h, G, off=poff, lens=plen_h):#018x}" == dg["parity"]
    assert f"{OC.group_digest(out_h, G, off=poff, lens=plen_h):#018x}" == dg["recovered"]
