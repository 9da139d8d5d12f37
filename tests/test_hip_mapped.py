"""GPU parity tests of QFEC_PTR_MAPPED: the FEC kernels read and write payloads
in pinned host memory in place (zero-copy over PCIe), index arrays staged by
the call.  Bit-exact against the oracle and the golden fixtures."""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC
from oracle import qfec_np as Q
from libquic_amd import qfec

from test_hip_ragged import run_ragged, sub, synth_batch

pytestmark = pytest.mark.gpu


def pinned(a):
    """a copy of `a` in qfec_host_alloc memory (kept alive by the returned buffer)"""
    hb = qfec.HostBuffer(max(1, a.nbytes))
    hb.array[:a.nbytes] = np.ascontiguousarray(a).view(np.uint8).ravel()
    return hb


@pytest.mark.parametrize("alloc", ["qfec_host_alloc", "torch_pin_memory"])
def test_fixed_mapped(ctx, alloc):
    k, L, n = 10, 1350, 9_001
    rows = OC.synth_fixed(Q.SEED_FIXED, 0, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    if alloc == "qfec_host_alloc":
        h_rows, h_par, h_out = pinned(rows), qfec.HostBuffer(n * L), qfec.HostBuffer(n * L)
        r, p, o = h_rows.array, h_par.array, h_out.array
    else:
        r = torch.from_numpy(rows).pin_memory()
        p = torch.zeros(n * L, dtype=torch.uint8).pin_memory()
        o = torch.zeros(n * L, dtype=torch.uint8).pin_memory()
    ctx.encode(r, k, L, n, p, mapped=True)
    ctx.recover(r, p, miss, k, L, n, o, mapped=True)
    par = p if isinstance(p, np.ndarray) else p.numpy()
    out = o if isinstance(o, np.ndarray) else o.numpy()
    assert np.array_equal(par, want_p)
    assert np.array_equal(out.reshape(n, L), rows.reshape(n, k, L)[np.arange(n), miss])


def test_fixed_mapped_strided(ctx):
    k, L, n = 5, 1350, 3000
    rs, ps = 1408, 1452
    rows = OC.synth_fixed(4, 0, n, k, L, row_stride=rs, group_stride=k * rs)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n, rs, k * rs, ps)
    h_rows, h_par, h_out = pinned(rows), qfec.HostBuffer(n * ps), qfec.HostBuffer(n * ps)
    h_par.array[:] = 0
    ctx.encode(h_rows.array, k, L, n, h_par.array, row_stride=rs, group_stride=k * rs,
               parity_stride=ps, mapped=True)
    assert np.array_equal(h_par.array, want_p)
    ctx.recover(h_rows.array, h_par.array, miss, k, L, n, h_out.array, row_stride=rs,
                group_stride=k * rs, parity_stride=ps, out_stride=ps, mapped=True)
    o = h_out.array.reshape(n, ps)[:, :L]
    assert np.array_equal(o, rows.reshape(n, k, rs)[np.arange(n), miss, :L])


def run_ragged_mapped(ctx, z):
    return run_ragged(ctx, z, host="mapped")


@pytest.mark.parametrize("tag", ["main", "tiny"])
def test_golden_ragged_mapped(ctx, golden_ragged, tag):
    z = sub(golden_ragged, tag)
    par, plen, out = run_ragged_mapped(ctx, z)
    assert np.array_equal(plen, z["parity_len"])
    assert np.array_equal(par, z["parity"])
    assert np.array_equal(out, z["recovered"])


def test_ragged_mapped_vs_oracle(ctx):
    n = 20_000
    ks, ptr, ln, off = synth_batch(n, g0=5)
    total = int(off[-1] + ln[-1])
    data = np.random.default_rng(11).integers(0, 256, total, dtype=np.uint8)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1452)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(5, 5 + n), ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1452)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1452)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged_mapped(ctx, z)
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


def test_xor_into_mapped(ctx):
    n = 1_000_003
    rng = np.random.default_rng(5)
    a, b = rng.integers(0, 256, n, dtype=np.uint8), rng.integers(0, 256, n, dtype=np.uint8)
    ha, hb = pinned(a), pinned(b)
    ctx.xor_into(ha.array, n, hb.array, mapped=True)
    assert np.array_equal(hb.array[:n], a ^ b)


def test_mapped_refuses_pageable_and_bad_flags(ctx):
    k, L, n = 3, 64, 4
    rows = np.zeros(n * k * L, np.uint8)  # pageable numpy memory
    par = qfec.HostBuffer(n * L)
    with pytest.raises(qfec.QfecError, match="QFEC_PTR_MAPPED"):
        ctx.encode(rows, k, L, n, par.array, mapped=True)
    h_rows = pinned(rows)
    with pytest.raises(qfec.QfecError, match="exclusive"):
        ctx.encode(h_rows.array, k, L, n, par.array, mapped=True, host=True)
    with pytest.raises(qfec.InvalidFecData):
        ctx.recover(h_rows.array, par.array, np.array([0, 1, 3, 0], np.uint8), k, L, n,
                    par.array, mapped=True)
    # ragged: an invalid length is reported before any device work
    ptr = np.array([0, 2], np.uint32)
    off = np.array([0, 100], np.uint64)
    ln = np.array([64, 1453], np.uint16)
    plen = np.zeros(1, np.uint16)
    with pytest.raises(qfec.InvalidFecData):
        ctx.encode_ragged(h_rows.array, off, ln, ptr, 1, par.array,
                          np.zeros(1, np.uint64), plen, mapped=True)


@pytest.mark.parametrize("chunk", ["7", "1000"])
def test_mapped_multi_chunk(ctx, chunk, monkeypatch):
    """QFEC_CHUNK_GROUPS shrinks the mapped paths' chunks: the table staging /
    lost-slot staging pipeline over several slots, against the oracle."""
    monkeypatch.setenv("QFEC_CHUNK_GROUPS", chunk)
    n = 3001
    ks, ptr, ln, off = synth_batch(n, g0=9)
    data = np.random.default_rng(int(chunk)).integers(0, 256, int(off[-1] + ln[-1]),
                                                      dtype=np.uint8)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1452)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(9, 9 + n), ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1452)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1452)
    assert rc == 0 and rc2 == 0
    z = dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
             out_off=poff, parity=want_p, recovered=want_o)
    par, plen, out = run_ragged(ctx, z, host="mapped")
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)
    # fixed shape: the lost-slot indices staged in chunks
    k, L, nf = 4, 200, 2003
    rows = OC.synth_fixed(Q.SEED_FIXED, 0, nf, k, L)
    mf = Q.drop_index(Q.SEED_DROP, np.arange(nf), k).astype(np.uint8)
    h_rows, h_par, h_out = pinned(rows), qfec.HostBuffer(nf * L), qfec.HostBuffer(nf * L)
    ctx.encode(h_rows.array, k, L, nf, h_par.array, mapped=True)
    ctx.recover(h_rows.array, h_par.array, mf, k, L, nf, h_out.array, mapped=True)
    _, want_pf = OC.encode_fixed(rows, k, L, nf)
    assert np.array_equal(h_par.array, want_pf)
    assert np.array_equal(h_out.array.reshape(nf, L), rows.reshape(nf, k, L)[np.arange(nf), mf])


def _mapped_case(n, g0, kmin=1, kmax=80, lmin=1, lmax=1452, seed=3):
    """a ragged batch with the latency kernel's edge shapes: k = 1, groups of more
    than 64 received packets and packets shorter than 16 B (both run the
    per-group fallback inside ragged_window_kernel), full-length packets."""
    ks, ptr, ln, off = synth_batch(n, kmin=kmin, kmax=kmax, lmin=lmin, lmax=lmax, g0=g0)
    data = np.random.default_rng(seed).integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    poff = np.arange(n, dtype=np.uint64) * np.uint64(1452)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(g0, g0 + n), ks).astype(np.uint8)
    rc, want_p, want_l = OC.encode_ragged(data, off, ln, ptr, poff, n * 1452)
    rc2, want_o = OC.recover_ragged(data, off, ln, ptr, want_p, poff, want_l, miss, poff,
                                    n * 1452)
    assert rc == 0 and rc2 == 0
    return dict(data=data, pkt_off=off, pkt_len=ln, grp_ptr=ptr, parity_off=poff, missing=miss,
                out_off=poff, parity=want_p, recovered=want_o), want_l


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257])
@pytest.mark.parametrize("shape", ["wide", "short", "full"])
def test_ragged_mapped_latency_path(ctx, n, shape):
    """<= 256 groups: tables read in place, ragged_window_kernel, completion by
    the host-mapped flag (257: the staged path); bit-exact vs the oracle."""
    kw = {"wide": {}, "short": dict(kmin=2, kmax=12, lmin=1, lmax=40),
          "full": dict(kmin=10, kmax=10, lmin=1452, lmax=1452)}[shape]
    z, want_l = _mapped_case(n, g0=1000 + n, **kw)
    par, plen, out = run_ragged(ctx, z, host="mapped")
    assert np.array_equal(plen, want_l)
    assert np.array_equal(par, z["parity"])
    assert np.array_equal(out, z["recovered"])


def test_ragged_mapped_latency_repeated(ctx):
    """many consecutive small flushes on one context (the completion token
    advances every call; a stale flag must never release a later call)"""
    z, want_l = _mapped_case(8, g0=77, kmin=3, kmax=12, lmin=16, lmax=1350)
    for _ in range(200):
        par, plen, out = run_ragged(ctx, z, host="mapped")
        assert np.array_equal(plen, want_l)
        assert np.array_equal(par, z["parity"])
        assert np.array_equal(out, z["recovered"])


def _page_aligned(a):
    """a copy of `a` in its own whole pages (two registrations never share a page)"""
    a = np.ascontiguousarray(a)
    n = max(a.nbytes, 1)
    raw = np.zeros(n + 2 * 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    view = raw[off:off + (n + 4095) // 4096 * 4096]
    out = view[:a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out  # a view: it keeps `raw` alive


def test_registered_host_memory(ctx):
    """qfec_host_register: an application's own host buffers (numpy arrays here),
    pinned and device-mapped in place, used by the mapped fixed and ragged
    paths; bit-exact vs the oracle; unregistered afterwards."""
    k, L, n = 10, 1350, 3001
    rows = _page_aligned(OC.synth_fixed(Q.SEED_FIXED, 0, n, k, L))
    par = _page_aligned(np.zeros(n * L, np.uint8))
    out = _page_aligned(np.zeros(n * L, np.uint8))
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    with qfec.HostRegistration(rows), qfec.HostRegistration(par), qfec.HostRegistration(out):
        ctx.encode(rows, k, L, n, par, mapped=True)
        ctx.recover(rows, par, miss, k, L, n, out, mapped=True)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out.reshape(n, L), rows.reshape(n, k, L)[np.arange(n), miss])
    # ragged, small (latency path) and large (staged tables)
    for m in (40, 3000):
        z, want_l = _mapped_case(m, g0=4242 + m, kmin=2, kmax=14, lmin=1, lmax=1452)
        data = _page_aligned(z["data"])
        p = _page_aligned(np.zeros(z["parity"].size, np.uint8))
        o = _page_aligned(np.zeros(z["recovered"].size, np.uint8))
        plen = np.zeros(m, np.uint16)
        with qfec.HostRegistration(data), qfec.HostRegistration(p), qfec.HostRegistration(o):
            ctx.encode_ragged(data, z["pkt_off"], z["pkt_len"], z["grp_ptr"], m, p,
                              z["parity_off"], plen, mapped=True)
            ctx.recover_ragged(data, z["pkt_off"], z["pkt_len"], z["grp_ptr"], m, p,
                               z["parity_off"], plen, z["missing"], o, z["out_off"], mapped=True)
        assert np.array_equal(plen, want_l)
        assert np.array_equal(p, z["parity"])
        assert np.array_equal(o, z["recovered"])
    # unregistered pageable memory is refused again
    with pytest.raises(qfec.QfecError, match="QFEC_PTR_MAPPED"):
        ctx.encode(rows, k, L, n, par, mapped=True)


@pytest.mark.parametrize("n", [3, 256, 2000])
def test_ragged_mapped_async(ctx, n):
    """QFEC_ASYNC (the event-loop form): an encode and a recover are queued on
    one context without waiting (n <= 256: the flag-completed latency path;
    2000: the block kernel, also reading its tables in place and signalling
    through the flag since round 4), polled with qfec_complete(wait=0), then
    completed; the outputs — bytes and the encode lengths, which arrive only
    at completion — equal the oracle's, and equal a synchronous call's."""
    z, want_l = _mapped_case(n, g0=4000 + n, kmin=2, kmax=40, lmin=1, lmax=1452)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(n * 1452)
    par.array[:] = 0xA5
    par_in = qfec.HostBuffer(n * 1452)
    par_in.array[:] = z["parity"]
    out = qfec.HostBuffer(n * 1452)
    out.array[:] = 0x5A
    plen = np.zeros(n, dtype=np.uint16)
    try:
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        ctx.recover_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n,
                           par_in.array, z["parity_off"], want_l, z["missing"], out.array,
                           z["out_off"], mapped=True, async_=True)
        polls = 0
        while ctx.complete(wait=False) == qfec.QFEC_PENDING:
            polls += 1
            assert polls < 10_000_000
        assert ctx.complete(wait=True) == 0  # nothing left: returns at once
        assert np.array_equal(plen, want_l)
        for g in range(n):
            o, m = int(z["parity_off"][g]), int(want_l[g])
            assert np.array_equal(par.array[o:o + m], z["parity"][o:o + m]), g
            assert np.array_equal(out.array[o:o + m], z["recovered"][o:o + m]), g
        # a synchronous call after async ones completes them first; same bytes
        plen2 = np.zeros(n, dtype=np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, out.array,
                          z["parity_off"], plen2, mapped=True)
        assert np.array_equal(plen, want_l) and np.array_equal(plen2, want_l)
    finally:
        for b in (data, par, par_in, out):
            b.close()


def test_ragged_mapped_async_error_at_completion(ctx):
    """An invalid batch refused by the host-side checks fails at the call
    (nothing queued); a valid async call after it completes normally."""
    z, want_l = _mapped_case(4, g0=9000, kmin=2, kmax=5, lmin=20, lmax=100)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(4 * 1452)
    plen = np.zeros(4, dtype=np.uint16)
    bad_len = z["pkt_len"].copy()
    bad_len[0] = 1453
    try:
        with pytest.raises(qfec.InvalidFecData):
            ctx.encode_ragged(data.array, z["pkt_off"], bad_len, z["grp_ptr"], 4, par.array,
                              z["parity_off"], plen, mapped=True, async_=True)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], 4, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        assert ctx.complete(wait=True) == 0
        assert np.array_equal(plen, want_l)
    finally:
        data.close()
        par.close()


@pytest.mark.parametrize("n", [3, 2000])
def test_ragged_mapped_async_tickets(ctx, n):
    """Each QFEC_ASYNC op completes on its own ticket (one
    Pending's completion no longer finishes and reports another's): tickets
    complete in any order, a synchronous call in between retires the queued
    ops but keeps their codes for their tickets, a completed ticket is
    unknown afterwards, and the outputs are the oracle's."""
    z, want_l = _mapped_case(n, g0=7000 + n, kmin=2, kmax=30, lmin=1, lmax=1452)
    data = qfec.HostBuffer(len(z["data"]))
    data.array[:] = z["data"]
    par = qfec.HostBuffer(n * 1452)
    par_in = qfec.HostBuffer(n * 1452)
    par_in.array[:] = z["parity"]
    out = qfec.HostBuffer(n * 1452)
    plen = np.zeros(n, dtype=np.uint16)
    try:
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        te = ctx.async_ticket()
        ctx.recover_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n,
                           par_in.array, z["parity_off"], want_l, z["missing"], out.array,
                           z["out_off"], mapped=True, async_=True)
        tr = ctx.async_ticket()
        assert te and tr and te != tr
        assert ctx.complete_ticket(tr) == 0   # the later op first
        assert ctx.complete_ticket(te) == 0
        assert np.array_equal(plen, want_l)
        for g in range(n):
            o, m = int(z["parity_off"][g]), int(want_l[g])
            assert np.array_equal(par.array[o:o + m], z["parity"][o:o + m]), g
            assert np.array_equal(out.array[o:o + m], z["recovered"][o:o + m]), g
        with pytest.raises(qfec.QfecError, match="ticket"):
            ctx.complete_ticket(te)
        # queued, then retired by a synchronous call: the code stays claimable
        plen[:] = 0
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, par.array,
                          z["parity_off"], plen, mapped=True, async_=True)
        t3 = ctx.async_ticket()
        plen2 = np.zeros(n, dtype=np.uint16)
        ctx.encode_ragged(data.array, z["pkt_off"], z["pkt_len"], z["grp_ptr"], n, out.array,
                          z["parity_off"], plen2, mapped=True)
        assert ctx.async_ticket() == 0  # the synchronous call queued nothing
        assert np.array_equal(plen, want_l) and np.array_equal(plen2, want_l)
        assert ctx.complete_ticket(t3) == 0
        assert ctx.complete(wait=True) == 0
    finally:
        for b in (data, par, par_in, out):
            b.close()
