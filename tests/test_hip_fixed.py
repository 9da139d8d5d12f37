"""GPU parity tests of the fixed-shape HIP path ([G][k][L] rows), through the C-ABI.

Every test compares the HIP kernels with the oracle (oracle/, CPU restatement)
or the golden fixtures bit-exactly; at BASELINE.json's full size (1M groups x
10 x 1350 B) it uses size-independent properties: the committed
checksum-of-checksums of the parity and of the revived rows, the
encode -> erase -> recover round trip, and parity XOR all rows == 0.
Parity is unpinned by the reference (no FEC source/vectors in the snapshot).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import oracle_c as OC
from oracle import qfec_np as Q
from libquic_amd import qfec

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a: np.ndarray, pad: int = 0, shift: int = 0) -> torch.Tensor:
    """Copy to the device; with `shift` the data starts `shift` bytes into the allocation."""
    flat = np.ascontiguousarray(a).view(np.uint8).ravel()
    t = torch.zeros(flat.size + pad + shift, dtype=torch.uint8, device=DEV)
    t[shift:shift + flat.size] = torch.from_numpy(flat).to(DEV)
    return t[shift:shift + flat.size] if not pad else t[shift:]


def host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy()


def run_fixed(ctx, rows_np, k, L, n, missing_np, shift=0, **kw):
    rows = dev(rows_np, shift=shift)
    par = torch.zeros(n * L + shift, dtype=torch.uint8, device=DEV)[shift:]
    ctx.encode(rows, k, L, n, par, **kw)
    ctx.sync()
    miss = dev(missing_np.astype(np.uint8))
    out = torch.zeros(n * L + shift, dtype=torch.uint8, device=DEV)[shift:]
    ctx.recover(rows, par, miss, k, L, n, out, **kw)
    ctx.sync()
    return host(par), host(out)


def test_golden_headline(ctx, golden_fixed):
    z = golden_fixed
    n, k, L = z["rows"].shape
    par, out = run_fixed(ctx, z["rows"], k, L, n, z["missing"])
    assert np.array_equal(par.reshape(n, L), z["parity"])
    assert np.array_equal(out.reshape(n, L), z["recovered"])


def test_golden_shapes(ctx, golden_shapes):
    tags = sorted({t.rsplit("_", 1)[0] for t in golden_shapes})
    for tag in tags:
        rows = golden_shapes[f"{tag}_rows"]
        n, k, L = rows.shape
        par, out = run_fixed(ctx, rows, k, L, n, golden_shapes[f"{tag}_missing"])
        assert np.array_equal(par.reshape(n, L), golden_shapes[f"{tag}_parity"]), tag
        assert np.array_equal(out.reshape(n, L), golden_shapes[f"{tag}_recovered"]), tag


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 9, 10, 11, 16, 17, 33, 255])
@pytest.mark.parametrize("L", [1, 7, 15, 16, 17, 31, 100, 1350, 1452])
def test_vs_oracle_k_L(ctx, k, L):
    n = 7 if k < 100 else 2
    rows = OC.synth_fixed(0xABC + k, 11, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(11, 11 + n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    _, want_o = OC.recover_fixed(rows, want_p, miss, k, L, n)
    par, out = run_fixed(ctx, rows, k, L, n, miss)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out, want_o)


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 8, 13])
def test_unaligned_buffers(ctx, shift):
    k, L, n = 10, 1350, 50
    rows = OC.synth_fixed(Q.SEED_FIXED, 0, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    par, out = run_fixed(ctx, rows, k, L, n, miss, shift=shift)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out.reshape(n, L), rows.reshape(n, k, L)[np.arange(n), miss])


def test_cached_policy_same_result(ctx):
    k, L, n = 10, 1350, 300
    rows = OC.synth_fixed(3, 0, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    p1, o1 = run_fixed(ctx, rows, k, L, n, miss)
    p2, o2 = run_fixed(ctx, rows, k, L, n, miss, cached=True)
    assert np.array_equal(p1, p2) and np.array_equal(o1, o2)


@pytest.mark.parametrize("row_stride,parity_stride", [(1360, 1350), (1408, 1408), (1350, 1452)])
def test_strided_padding_study_layouts(ctx, row_stride, parity_stride):
    k, L, n = 10, 1350, 64
    gs = k * row_stride
    rows = OC.synth_fixed(Q.SEED_FIXED, 0, n, k, L, row_stride=row_stride, group_stride=gs)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n, row_stride, gs, parity_stride)
    _, want_o = OC.recover_fixed(rows, want_p, miss, k, L, n, row_stride, gs, parity_stride,
                                 parity_stride)
    d_rows = dev(rows)
    d_par = torch.zeros(n * parity_stride, dtype=torch.uint8, device=DEV)
    ctx.encode(d_rows, k, L, n, d_par, row_stride=row_stride, group_stride=gs,
               parity_stride=parity_stride)
    d_out = torch.zeros(n * parity_stride, dtype=torch.uint8, device=DEV)
    ctx.recover(d_rows, d_par, dev(miss), k, L, n, d_out, row_stride=row_stride,
                group_stride=gs, parity_stride=parity_stride, out_stride=parity_stride)
    ctx.sync()
    par = host(d_par).reshape(n, parity_stride)
    out = host(d_out).reshape(n, parity_stride)
    assert np.array_equal(par[:, :L], want_p.reshape(n, parity_stride)[:, :L])
    assert not par[:, L:].any()  # padding bytes untouched
    assert np.array_equal(out[:, :L], want_o.reshape(n, parity_stride)[:, :L])


def test_device_synth_matches_oracle(ctx):
    for (k, L, g0, n) in [(10, 1350, 0, 5), (10, 1350, 1_000_000, 3), (3, 17, 9, 4),
                          (255, 64, 2, 1), (2, 5, 0, 3)]:
        t = torch.zeros(n * k * L, dtype=torch.uint8, device=DEV)
        ctx.synth_fixed(t, k, L, g0, n, Q.SEED_FIXED)
        assert np.array_equal(host(t), OC.synth_fixed(Q.SEED_FIXED, g0, n, k, L))


def test_device_synth_many_rows(ctx):
    """More than 2^24 rows: several synth launches (a dispatch's grid is at most
    2^32 work-items); sampled groups, the first and the last, vs the oracle."""
    k, L, n = 5, 17, 4_000_000
    t = torch.zeros(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(t, k, L, 0, n, Q.SEED_FIXED)
    h = host(t)
    for g in [0, 3_355_443, 3_355_444, n - 1] + list(np.random.default_rng(3).choice(n, 16)):
        g = int(g)
        assert np.array_equal(h[g * k * L:(g + 1) * k * L],
                              OC.synth_fixed(Q.SEED_FIXED, g, 1, k, L)), g


def test_errors(ctx):
    t = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    with pytest.raises(qfec.InvalidFecData):
        ctx.encode(t, 0, 100, 1, t)          # k = 0
    with pytest.raises(qfec.InvalidFecData):
        ctx.encode(t, 256, 2, 1, t)          # k > 255
    with pytest.raises(qfec.InvalidFecData):
        ctx.encode(t, 1, 1453, 1, t)         # L > kMaxPacketSize
    with pytest.raises(qfec.InvalidFecData):
        ctx.encode(t, 2, 100, 1, t, row_stride=50)  # stride < L
    # device-detected: missing index >= k latches QUIC_INVALID_FEC_DATA at sync;
    # the other groups are still revived, the bad group's output is untouched
    k, L, n = 4, 64, 3
    rows = OC.synth_fixed(1, 0, n, k, L)
    _, p = OC.encode_fixed(rows, k, L, n)
    miss = np.array([1, 9, 2], dtype=np.uint8)
    out = torch.full((n * L,), 0xEE, dtype=torch.uint8, device=DEV)
    ctx.recover(dev(rows), dev(p), dev(miss), k, L, n, out)
    with pytest.raises(qfec.InvalidFecData):
        ctx.sync()
    ctx.sync()  # error cleared
    o = host(out).reshape(n, L)
    r = rows.reshape(n, k, L)
    assert np.array_equal(o[0], r[0, 1]) and np.array_equal(o[2], r[2, 2])
    assert (o[1] == 0xEE).all()
    assert ctx.encode(t, 3, 10, 0, t) == 0  # empty batch is fine


@pytest.mark.parametrize("pinned", [False, True])
def test_host_pointer_path(ctx, pinned):
    # several staging chunks (64 MiB / 13500 B = 4971 groups per chunk)
    k, L, n = 10, 1350, 12_001
    rows = OC.synth_fixed(Q.SEED_FIXED, 0, n, k, L)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    if pinned:
        h_rows = torch.from_numpy(rows).pin_memory()
        h_par = torch.zeros(n * L, dtype=torch.uint8).pin_memory()
        h_out = torch.zeros(n * L, dtype=torch.uint8).pin_memory()
        ctx.encode(h_rows, k, L, n, h_par, host=True)
        ctx.recover(h_rows, h_par, miss, k, L, n, h_out, host=True)
        par, out = h_par.numpy(), h_out.numpy()
    else:
        par = np.zeros(n * L, np.uint8)
        out = np.zeros(n * L, np.uint8)
        ctx.encode(rows, k, L, n, par, host=True)
        ctx.recover(rows, par, miss, k, L, n, out, host=True)
    assert np.array_equal(par, want_p)
    assert np.array_equal(out.reshape(n, L), rows.reshape(n, k, L)[np.arange(n), miss])


def test_host_pointer_strided(ctx):
    k, L, n = 5, 1350, 6000
    rs, ps = 1408, 1452
    rows = OC.synth_fixed(4, 0, n, k, L, row_stride=rs, group_stride=k * rs)
    miss = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    _, want_p = OC.encode_fixed(rows, k, L, n, rs, k * rs, ps)
    par = np.zeros(n * ps, np.uint8)
    ctx.encode(rows, k, L, n, par, row_stride=rs, group_stride=k * rs, parity_stride=ps,
               host=True)
    assert np.array_equal(par, want_p)
    out = np.zeros(n * ps, np.uint8)
    ctx.recover(rows, par, miss, k, L, n, out, row_stride=rs, group_stride=k * rs,
                parity_stride=ps, out_stride=ps, host=True)
    o = out.reshape(n, ps)[:, :L]
    assert np.array_equal(o, rows.reshape(n, k, rs)[np.arange(n), miss, :L])


def test_host_invalid_missing(ctx):
    rows = np.zeros(3 * 10, np.uint8)
    with pytest.raises(qfec.InvalidFecData):
        ctx.recover(rows, np.zeros(10, np.uint8), np.array([3], np.uint8), 3, 10, 1,
                    np.zeros(10, np.uint8), host=True)


def test_torch_stream(ctx):
    s = torch.cuda.Stream()
    k, L, n = 10, 1350, 1000
    rows = OC.synth_fixed(8, 0, n, k, L)
    _, want_p = OC.encode_fixed(rows, k, L, n)
    d_rows = dev(rows)
    par = torch.zeros(n * L, dtype=torch.uint8, device=DEV)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        ctx.set_stream(s)
        ctx.encode(d_rows, k, L, n, par)
        res = par.cpu()  # ordered on s
    # back to the session's setting (conftest: torch's current stream), so later
    # tests' torch fills stay ordered with the context's launches
    ctx.set_stream(torch.cuda.current_stream())
    s.synchronize()
    assert np.array_equal(res.numpy(), want_p)


def test_full_size_headline(ctx):
    """BASELINE configs[1]/[2] at full size: 1M groups x 10 x 1350 B, device-resident."""
    with open(os.path.join(GOLDEN, "full_digests.json")) as f:
        dg = json.load(f)["digests"]["g0=0,n=1048576"]
    k, L, n = 10, 1350, 1 << 20
    rows = torch.empty(n * k * L, dtype=torch.uint8, device=DEV)
    ctx.synth_fixed(rows, k, L, 0, n, Q.SEED_FIXED)
    par = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.encode(rows, k, L, n, par)
    miss_np = Q.drop_index(Q.SEED_DROP, np.arange(n), k).astype(np.uint8)
    miss = torch.from_numpy(miss_np).to(DEV)
    out = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    ctx.recover(rows, par, miss, k, L, n, out)
    ctx.sync()
    torch.cuda.synchronize()
    # 1) checksum of checksums vs the committed oracle digests
    par_h = par.cpu().numpy()
    out_h = out.cpu().numpy()
    assert f"{OC.group_digest(par_h, n, L, L):#018x}" == dg["parity"]
    assert f"{OC.group_digest(out_h, n, L, L):#018x}" == dg["recovered"]
    # 2) round trip on the device: revived row == erased row, every group
    r3 = rows.view(n, k, L)
    lost = r3[torch.arange(n, device=DEV), miss.long()]
    assert torch.equal(lost, out.view(n, L))
    # 3) parity XOR every row == 0
    acc = par.view(n, L).clone()
    for i in range(k):
        acc ^= r3[:, i]
    assert not bool(acc.any())
    # 4) sampled groups byte-exact vs the oracle
    rng = np.random.default_rng(1)
    for g in rng.choice(n, 64, replace=False):
        rr = OC.synth_fixed(Q.SEED_FIXED, int(g), 1, k, L)
        _, pp = OC.encode_fixed(rr, k, L, 1)
        assert np.array_equal(par_h[g * L:(g + 1) * L], pp)


def test_xor_into(ctx):
    rng = np.random.default_rng(5)
    for n in [1, 15, 16, 17, 1350, 100_003]:
        for shift in [0, 3]:
            a = rng.integers(0, 256, n, dtype=np.uint8)
            b = rng.integers(0, 256, n, dtype=np.uint8)
            da, db = dev(a, shift=shift), dev(b, shift=(shift * 2) % 7)
            ctx.xor_into(da, n, db)
            ctx.sync()
            assert np.array_equal(host(db), a ^ b)
            hb = b.copy()
            ctx.xor_into(a, n, hb, host=True)
            assert np.array_equal(hb, a ^ b)


def test_xor_into_host_scratch_reuse(ctx):
    """Host-pointer calls run on the context's grow-only device scratch:
    growing, shrinking and growing again sizes keep every result exact."""
    rng = np.random.default_rng(6)
    for n in [10, 3_000_001, 50, 17, 5_000_000, 1, 3_000_001]:
        a = rng.integers(0, 256, n, dtype=np.uint8)
        b = rng.integers(0, 256, n, dtype=np.uint8)
        hb = b.copy()
        ctx.xor_into(a, n, hb, host=True)
        assert np.array_equal(hb, a ^ b), n
