"""GPU parity tests of the packet-entropy kernels (qent_kernels.hip) through
the C-ABI (qfec_entropy_cumulative_batch / qfec_entropy_validate_batch): the
fixture the REFERENCE's QuicSentEntropyManager produced
(tests/golden/entropy.npz), the reference-pinned oracle (oracle/qent_oracle.c)
on random ragged batches, and a large batch checked through numpy's
bitwise_xor.accumulate.  Bit-exact."""
import numpy as np
import pytest
import torch

from libquic_amd import synth
from oracle import oracle_c as OC

from conftest import load_npz

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dv(a):
    a = np.ascontiguousarray(a)
    sig = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[a.dtype.itemsize]
    if a.size == 0:
        return torch.zeros(1, dtype=torch.uint8, device=DEV)
    if a.dtype.itemsize == 1:
        return torch.from_numpy(a.copy()).to(DEV)
    return torch.from_numpy(a.view(sig).copy()).to(DEV)


def run_gpu(ctx, d, host=False, mean_hint=None):
    n_conns = d["conn_ptr"].size - 1
    n_acks = d["ack_conn"].size
    if host:
        cum = np.zeros(max(d["entropy"].size, 1), np.uint8)
        ctx.entropy_cumulative(d["entropy"], d["conn_ptr"], d["cum_base"], n_conns, cum, host=True)
        ok = np.zeros(max(n_acks, 1), np.uint8)
        ctx.entropy_validate(cum, d["conn_ptr"], d["first_pn"], d["cum_base"], n_conns,
                             d["ack_conn"], d["largest"], d["claimed"], d["range_ptr"],
                             d["range_lo"] if d["range_lo"].size else None,
                             d["range_hi"] if d["range_hi"].size else None, n_acks, ok, host=True)
        return cum[:d["entropy"].size], ok[:n_acks]
    t = {k: dv(d[k]) for k in ("entropy", "conn_ptr", "first_pn", "cum_base", "ack_conn",
                               "largest", "claimed", "range_ptr", "range_lo", "range_hi")}
    cum = torch.zeros(max(d["entropy"].size, 1), dtype=torch.uint8, device=DEV)
    ok = torch.full((max(n_acks, 1),), 7, dtype=torch.uint8, device=DEV)
    hint = 0 if mean_hint is None else mean_hint * n_conns  # launch shape only
    ctx.entropy_cumulative(t["entropy"], t["conn_ptr"], t["cum_base"], n_conns, cum,
                           n_packets=hint)
    ctx.entropy_validate(cum, t["conn_ptr"], t["first_pn"], t["cum_base"], n_conns, t["ack_conn"],
                         t["largest"], t["claimed"], t["range_ptr"], t["range_lo"], t["range_hi"],
                         n_acks, ok)
    ctx.sync()
    return cum.cpu().numpy()[:d["entropy"].size], ok.cpu().numpy()[:n_acks]


def oracle(d):
    cum = OC.entropy_cumulative_batch(d["entropy"], d["conn_ptr"], d["cum_base"])
    ok = OC.entropy_validate_batch(cum, d["conn_ptr"], d["first_pn"], d["cum_base"],
                                   d["ack_conn"], d["largest"], d["claimed"], d["range_ptr"],
                                   d["range_lo"], d["range_hi"])
    return cum, ok


@pytest.mark.parametrize("host", [False, True])
def test_reference_fixture(ctx, host):
    g = load_npz("entropy.npz")
    cum, ok = run_gpu(ctx, g, host=host)
    assert np.array_equal(cum, g["ref_cum"])
    assert np.array_equal(ok, g["ref_ok"])


@pytest.mark.parametrize("mean_hint", [None, 100, 200, 400, 1000])  # 8/16/32/64 lanes/conn
@pytest.mark.parametrize("seed,max_packets", [(11, 50), (12, 700), (13, 3000)])
def test_random_ragged_vs_oracle(ctx, seed, max_packets, mean_hint):
    rng = np.random.default_rng(seed)
    d = synth.entropy_batch(rng, 257, max_packets=max_packets, acks_per_conn=3, max_ranges=5)
    cum, ok = run_gpu(ctx, d, mean_hint=mean_hint)
    rc, rok = oracle(d)
    assert np.array_equal(cum, rc)
    assert np.array_equal(ok, rok)
    assert 0 < int(ok.sum()) < ok.size


def test_large_batch_accumulate(ctx):
    """2^18 connections x 128-packet windows: cum == numpy's per-row
    bitwise_xor.accumulate ^ base; one ack per connection with its true hash
    (valid) and one corrupted (invalid)."""
    C, W = 1 << 18, 128
    rng = np.random.default_rng(5)
    pn0 = rng.integers(1, 1 << 30, C).astype(np.uint64)
    flags = rng.integers(0, 2, (C, W)).astype(np.uint8)
    pns = pn0[:, None] + np.arange(W, dtype=np.uint64)[None, :]
    e = (flags << (pns % np.uint64(8)).astype(np.uint8)).astype(np.uint8)
    base = rng.integers(0, 256, C).astype(np.uint8)
    want = np.bitwise_xor.accumulate(e, axis=1) ^ base[:, None]
    d = {"entropy": e.reshape(-1), "conn_ptr": (np.arange(C + 1, dtype=np.uint64) * W),
         "first_pn": pn0, "cum_base": base}
    largest = pn0 + rng.integers(0, W, C).astype(np.uint64)
    true = want[np.arange(C), (largest - pn0).astype(np.int64)]
    d["ack_conn"] = np.concatenate([np.arange(C), np.arange(C)]).astype(np.uint32)
    d["largest"] = np.concatenate([largest, largest])
    d["claimed"] = np.concatenate([true, true ^ np.uint8(0x5A)]).astype(np.uint8)
    d["range_ptr"] = np.zeros(2 * C + 1, np.uint32)
    d["range_lo"] = np.zeros(0, np.uint64)
    d["range_hi"] = np.zeros(0, np.uint64)
    cum, ok = run_gpu(ctx, d, mean_hint=W)
    assert np.array_equal(cum, want.reshape(-1))
    assert ok[:C].all() and not ok[C:].any()


def test_defined_edges(ctx):
    d = {"entropy": np.array([1, 2, 4], np.uint8), "conn_ptr": np.array([0, 3, 3], np.uint64),
         "first_pn": np.array([5, 9], np.uint64), "cum_base": np.array([0x10, 0x20], np.uint8)}
    acks = [(0, 7, 0x17, [], 1), (0, 4, 0x10, [], 1), (0, 3, 0x10, [], 0), (0, 8, 0x17, [], 0),
            (0, 7, 0x17 ^ 2, [(6, 7)], 1), (0, 7, 0x17 ^ 6, [(6, 8)], 1),
            (0, 7, 0x17, [(7, 9)], 0), (0, 7, 0x17, [(4, 6)], 0), (0, 7, 0x17, [(6, 6)], 1),
            (1, 8, 0x20, [], 1), (1, 9, 0x20, [], 0), (2, 8, 0x20, [], 0)]
    d["ack_conn"] = np.array([a[0] for a in acks], np.uint32)
    d["largest"] = np.array([a[1] for a in acks], np.uint64)
    d["claimed"] = np.array([a[2] for a in acks], np.uint8)
    lo, hi, ptr = [], [], [0]
    for a in acks:
        for l, h in a[3]:
            lo.append(l)
            hi.append(h)
        ptr.append(len(lo))
    d["range_ptr"] = np.array(ptr, np.uint32)
    d["range_lo"] = np.array(lo, np.uint64)
    d["range_hi"] = np.array(hi, np.uint64)
    cum, ok = run_gpu(ctx, d)
    assert list(cum) == [0x11, 0x13, 0x17]
    assert list(ok) == [a[4] for a in acks]


def test_empty_calls(ctx):
    x = torch.zeros(8, dtype=torch.uint8, device=DEV)
    assert ctx.entropy_cumulative(x, x, None, 0, x) == 0
    assert ctx.entropy_validate(x, x, x, None, 0, x, x, x, x, x, x, 0, x) == 0
