"""GPU parity tests of the NULL packet-protection kernels (qpp_kernels.hip)
through the C-ABI (qfec_null_encrypt_batch / qfec_null_decrypt_batch) against
the fixtures the REFERENCE's NullEncrypter / NullDecrypter generated
(tests/golden/null_protect.npz) and the reference-pinned C oracle
(oracle/qpp_oracle.c).  Bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC

from conftest import load_npz

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TAG = 12


def dv(a):
    """device copy preserving bits (torch has no wide unsigned dtypes)"""
    a = np.ascontiguousarray(a)
    sig = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[a.dtype.itemsize]
    if a.dtype.itemsize == 1:
        return torch.from_numpy(a.copy()).to(DEV)
    return torch.from_numpy(a.view(sig).copy()).to(DEV)


def offsets(lens):
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    return off


@pytest.fixture(scope="module")
def gold():
    return load_npz("null_protect.npz")


def encrypt_dev(ctx, data, ad_off, ad_len, pt_off, pt_len, out_off, out_size, host=False):
    n = pt_len.size
    if host:
        out = np.zeros(out_size, np.uint8)
        ctx.null_encrypt(data, ad_off, ad_len, pt_off, pt_len, n, out, out_off, host=True)
        return out
    out = torch.zeros(out_size, dtype=torch.uint8, device=DEV)
    ctx.null_encrypt(dv(data), dv(ad_off), dv(ad_len), dv(pt_off), dv(pt_len), n, out,
                     dv(out_off))
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy()


def decrypt_dev(ctx, data, ad_off, ad_len, ct_off, ct_len, out_off, out_size, fill=0, host=False,
                scratch_out=False):
    n = ct_len.size
    if host:
        out = np.full(out_size, fill, np.uint8)
        ok = np.full(n, 7, np.uint8)
        ctx.null_decrypt(data, ad_off, ad_len, ct_off, ct_len, n, out, out_off, ok, host=True)
        return out, ok
    out = torch.full((out_size,), fill, dtype=torch.uint8, device=DEV)
    ok = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    ctx.null_decrypt(dv(data), dv(ad_off), dv(ad_len), dv(ct_off), dv(ct_len), n, out,
                     dv(out_off), ok, scratch_out=scratch_out)
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy(), ok.cpu().numpy()


@pytest.mark.parametrize("host", [False, True])
def test_encrypt_golden(ctx, gold, host):
    g = gold
    out_off = offsets(g["pt_len"].astype(np.uint64) + TAG)
    out = encrypt_dev(ctx, g["data"], g["ad_off"], g["ad_len"], g["pt_off"], g["pt_len"],
                      out_off, g["ct"].size, host=host)
    assert np.array_equal(out, g["ct"])


@pytest.mark.parametrize("host", [False, True])
def test_decrypt_golden(ctx, gold, host):
    g = gold
    plen = np.maximum(g["dec_ct_len"].astype(np.int64) - TAG, 0)
    out_off = offsets(plen)
    out, ok = decrypt_dev(ctx, g["dec_data"], g["dec_ad_off"], g["dec_ad_len"], g["dec_ct_off"],
                          g["dec_ct_len"], out_off, int(plen.sum()) + 1, fill=0xA5, host=host)
    assert np.array_equal(ok, g["dec_ok"])
    pos = 0
    for p in range(ok.size):
        seg = out[int(out_off[p]):int(out_off[p]) + int(plen[p])]
        if ok[p]:
            assert np.array_equal(seg, g["dec_pt"][pos:pos + seg.size]), p
            pos += seg.size
        else:  # output untouched on a failed tag (memcpy after the check)
            assert (seg == 0xA5).all(), p


def test_encrypt_in_place(ctx, gold):
    """QuicPacketCreator::EncryptInPlace layout: [header | payload | 12 spare];
    the output starts at the payload (tag there, payload shifted right)."""
    g = gold
    n = g["pt_len"].size
    rec = g["ad_len"].astype(np.uint64) + g["pt_len"].astype(np.uint64) + TAG
    base = offsets(rec)
    buf = np.zeros(int(rec.sum()), np.uint8)
    ad_off = base
    pt_off = base + g["ad_len"].astype(np.uint64)
    for p in range(n):
        a, l_ = int(g["ad_len"][p]), int(g["pt_len"][p])
        buf[int(ad_off[p]):int(ad_off[p]) + a] = g["data"][int(g["ad_off"][p]):int(g["ad_off"][p]) + a]
        buf[int(pt_off[p]):int(pt_off[p]) + l_] = g["data"][int(g["pt_off"][p]):int(g["pt_off"][p]) + l_]
    d = dv(buf)
    ctx.null_encrypt(d, dv(ad_off), dv(g["ad_len"]), dv(pt_off), dv(g["pt_len"]), n, d, dv(pt_off))
    ctx.sync()
    torch.cuda.synchronize()
    res = d.cpu().numpy()
    for p in range(n):
        c = g["ct"][int(g["ct_off"][p]):int(g["ct_off"][p]) + int(g["ct_len"][p])]
        assert np.array_equal(res[int(pt_off[p]):int(pt_off[p]) + c.size], c), p
        a = int(g["ad_len"][p])  # header untouched
        assert np.array_equal(res[int(ad_off[p]):int(ad_off[p]) + a],
                              g["data"][int(g["ad_off"][p]):int(g["ad_off"][p]) + a])


def random_batch(n, seed, lmax=1452):
    rng = np.random.default_rng(seed)
    ad_len = rng.integers(0, 48, n).astype(np.uint16)
    pt_len = rng.integers(0, lmax + 1, n).astype(np.uint16)
    # scattered records with gaps (unaligned offsets)
    gaps = rng.integers(0, 9, 2 * n).astype(np.uint64)
    lens = np.empty(2 * n, np.uint64)
    lens[0::2] = ad_len
    lens[1::2] = pt_len
    off = offsets(lens + gaps) + gaps
    data = rng.integers(0, 256, int(off[-1] + lens[-1]) + 1, dtype=np.uint8)
    return data, off[0::2].copy(), ad_len, off[1::2].copy(), pt_len


def test_encrypt_decrypt_random_vs_oracle(ctx):
    n = 40_000
    data, ad_off, ad_len, pt_off, pt_len = random_batch(n, 11)
    out_off = offsets(pt_len.astype(np.uint64) + TAG)
    size = int(out_off[-1]) + int(pt_len[-1]) + TAG
    got = encrypt_dev(ctx, data, ad_off, ad_len, pt_off, pt_len, out_off, size)
    want = OC.null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, out_off, size, threads=8)
    assert np.array_equal(got, want)
    # decrypt the device ciphertexts (headers re-used), with every 5th tampered
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)])
    h_off = offsets(ad_len.astype(np.uint64))
    ct = got.copy()
    ct_len = (pt_len.astype(np.uint64) + TAG).astype(np.uint16)
    flip = np.arange(0, n, 5)
    pos = out_off[flip] + (np.arange(flip.size) % (ct_len[flip].astype(np.uint64)))
    ct[pos.astype(np.int64)] ^= 0x40
    buf = np.concatenate([hdr, ct])
    ct_off = out_off + np.uint64(hdr.size)
    dout_off = offsets(pt_len.astype(np.uint64))
    out, ok = decrypt_dev(ctx, buf, h_off, ad_len, ct_off, ct_len, dout_off,
                          int(pt_len.astype(np.int64).sum()) + 1)
    want_out, want_ok = OC.null_decrypt_batch(buf, h_off, ad_len, ct_off, ct_len, dout_off,
                                              int(pt_len.astype(np.int64).sum()) + 1)
    assert np.array_equal(ok, want_ok)
    assert want_ok[flip].sum() == 0 and want_ok.sum() == n - flip.size
    good = np.repeat(ok.astype(bool), pt_len.astype(np.int64))
    assert np.array_equal(out[:good.size][good], want_out[:good.size][good])


@pytest.mark.parametrize("lmax", [0, 15, 16, 17])
def test_short_payloads(ctx, lmax):
    n = 3000
    data, ad_off, ad_len, pt_off, pt_len = random_batch(n, 20 + lmax, lmax=lmax)
    out_off = offsets(pt_len.astype(np.uint64) + TAG)
    size = int(out_off[-1]) + int(pt_len[-1]) + TAG
    got = encrypt_dev(ctx, data, ad_off, ad_len, pt_off, pt_len, out_off, size)
    want = OC.null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, out_off, size)
    assert np.array_equal(got, want)
    # and back: every head / tail split of the destination-aligned copy
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)])
    h_off = offsets(ad_len.astype(np.uint64))
    ct_len = (pt_len.astype(np.uint64) + TAG).astype(np.uint16)
    buf = np.concatenate([hdr, got])
    ct_off = out_off + np.uint64(hdr.size)
    dout_off = offsets(pt_len.astype(np.uint64)) + np.uint64(3)
    dsize = int(pt_len.astype(np.int64).sum()) + 4
    out, ok = decrypt_dev(ctx, buf, h_off, ad_len, ct_off, ct_len, dout_off, dsize)
    want_out, want_ok = OC.null_decrypt_batch(buf, h_off, ad_len, ct_off, ct_len, dout_off, dsize)
    assert ok.all() and np.array_equal(ok, want_ok)
    assert np.array_equal(out, want_out)


@pytest.mark.parametrize("seed", [1, 2])
def test_encrypt_in_place_random(ctx, seed):
    """EncryptInPlace on scattered records of random lengths: every alignment
    of the payload (and so of the destination, payload + 12) against the
    destination-aligned head / chunk / tail split."""
    rng = np.random.default_rng(100 + seed)
    n = 6000
    ad_len = rng.integers(0, 48, n).astype(np.uint16)
    pt_len = rng.integers(0, 1453, n).astype(np.uint16)
    gaps = rng.integers(0, 19, n).astype(np.uint64)
    rec = ad_len.astype(np.uint64) + pt_len.astype(np.uint64) + TAG + gaps
    ad_off = offsets(rec) + gaps
    pt_off = ad_off + ad_len.astype(np.uint64)
    size = int(ad_off[-1] + ad_len[-1] + pt_len[-1]) + TAG
    data = rng.integers(0, 256, size, dtype=np.uint8)
    want = OC.null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, pt_off, size)
    d = dv(data)
    ctx.null_encrypt(d, dv(ad_off), dv(ad_len), dv(pt_off), dv(pt_len), n, d, dv(pt_off))
    ctx.sync()
    torch.cuda.synchronize()
    res = d.cpu().numpy()
    for p in range(0, n, 7):
        o, c = int(pt_off[p]), int(pt_len[p]) + TAG
        assert np.array_equal(res[o:o + c], want[o:o + c]), p
    mask = np.zeros(size, bool)
    for o, c in zip(pt_off, pt_len.astype(np.int64) + TAG):
        mask[int(o):int(o) + int(c)] = True
    assert np.array_equal(res[mask], want[mask])
    assert np.array_equal(res[~mask], data[~mask])  # headers and gaps untouched


@pytest.mark.parametrize("lmax", [17, 1452])
def test_decrypt_scratch_output_one_pass(ctx, lmax):
    """QFEC_SCRATCH_OUTPUT: one pass over the ciphertext; ok[] as the oracle,
    verified packets' plaintext exact, and a failed packet's output is its
    unverified plaintext (the ciphertext after the tag), never anything else."""
    n = 20_000
    data, ad_off, ad_len, pt_off, pt_len = random_batch(n, 77 + lmax, lmax=lmax)
    out_off = offsets(pt_len.astype(np.uint64) + TAG)
    size = int(out_off[-1]) + int(pt_len[-1]) + TAG
    ct = OC.null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, out_off, size)
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)])
    h_off = offsets(ad_len.astype(np.uint64))
    ct_len = (pt_len.astype(np.uint64) + TAG).astype(np.uint16)
    flip = np.arange(0, n, 7)
    pos = out_off[flip] + (np.arange(flip.size) % (ct_len[flip].astype(np.uint64)))
    ct = ct.copy()
    ct[pos.astype(np.int64)] ^= 0x10
    buf = np.concatenate([hdr, ct])
    ct_off = out_off + np.uint64(hdr.size)
    dout_off = offsets(pt_len.astype(np.uint64)) + np.uint64(5)
    dsize = int(pt_len.astype(np.int64).sum()) + 6
    out, ok = decrypt_dev(ctx, buf, h_off, ad_len, ct_off, ct_len, dout_off, dsize, fill=0xA5,
                          scratch_out=True)
    want_out, want_ok = OC.null_decrypt_batch(buf, h_off, ad_len, ct_off, ct_len, dout_off, dsize)
    assert np.array_equal(ok, want_ok)
    assert want_ok[flip].sum() == 0 and want_ok.sum() == n - flip.size
    for p in range(n):
        o, l = int(dout_off[p]), int(pt_len[p])
        c = int(ct_off[p]) + TAG
        assert np.array_equal(out[o:o + l], buf[c:c + l]), p   # verified or not
    good = np.repeat(ok.astype(bool), pt_len.astype(np.int64))
    assert np.array_equal(out[5:5 + good.size][good], want_out[5:5 + good.size][good])
