"""GPU parity tests of the ChaCha20-Poly1305 packet-protection kernels
(qpp_kernels.hip) through the C-ABI (qfec_chacha20poly1305_seal/open_batch):
BoringSSL's own vectors from the reference tree (ciphertext + the 12-byte tag
prefix QUIC keeps) and random batches against the vector-pinned C oracle
(oracle/qaead_oracle.c).  Bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC

from conftest import load_npz

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TAG = 12


def dv(a):
    a = np.ascontiguousarray(a)
    if a.dtype.itemsize == 1:
        return torch.from_numpy(a.view(np.uint8).copy()).to(DEV)
    sig = {2: np.int16, 4: np.int32, 8: np.int64}[a.dtype.itemsize]
    return torch.from_numpy(a.view(sig).copy()).to(DEV)


def offsets(lens):
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    return off


def seal(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size,
         host=False):
    n = in_len.size
    if host:
        out = np.zeros(size, np.uint8)
        ctx.chacha20poly1305_seal(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len,
                                  n, out, out_off, host=True)
        return out
    out = torch.zeros(size, dtype=torch.uint8, device=DEV)
    ctx.chacha20poly1305_seal(dv(keys), dv(pre), dv(kidx), dv(pn),
                              None if path is None else dv(path), dv(data), dv(ad_off),
                              dv(ad_len), dv(in_off), dv(in_len), n, out, dv(out_off))
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy()


def open_(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size,
          host=False, fill=0xA5):
    n = in_len.size
    if host:
        out = np.full(size, fill, np.uint8)
        ok = np.full(n, 7, np.uint8)
        ctx.chacha20poly1305_open(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len,
                                  n, out, out_off, ok, host=True)
        return out, ok
    out = torch.full((size,), fill, dtype=torch.uint8, device=DEV)
    ok = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    ctx.chacha20poly1305_open(dv(keys), dv(pre), dv(kidx), dv(pn),
                              None if path is None else dv(path), dv(data), dv(ad_off),
                              dv(ad_len), dv(in_off), dv(in_len), n, out, dv(out_off), ok)
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy(), ok.cpu().numpy()


@pytest.mark.parametrize("host", [False, True])
def test_boringssl_vectors(ctx, host):
    z = load_npz("chacha20_poly1305.npz")
    n = z["key_len"].size

    def get(f, i):
        o, l = int(z[f + "_off"][i]), int(z[f + "_len"][i])
        return z[f][o:o + l]
    keys = np.concatenate([get("key", i) for i in range(n)])
    nonces = [get("nonce", i) for i in range(n)]
    pre = np.concatenate([x[:4] for x in nonces])
    pn = np.array([int.from_bytes(bytes(x[4:]), "little") for x in nonces], np.uint64)
    kidx = np.arange(n, dtype=np.uint32)
    ads = [get("ad", i) for i in range(n)]
    pts = [get("in", i) for i in range(n)]
    ad_len = np.array([a.size for a in ads], np.uint16)
    in_len = np.array([p.size for p in pts], np.uint16)
    data = np.concatenate(ads + pts + [np.zeros(1, np.uint8)])
    ad_off = offsets(ad_len)
    in_off = offsets(in_len) + np.uint64(int(ad_len.astype(np.int64).sum()))
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    size = int(in_len.astype(np.int64).sum()) + TAG * n
    out = seal(ctx, keys, pre, kidx, pn, None, data, ad_off, ad_len, in_off, in_len, out_off, size,
               host=host)
    checked_tags = 0
    for i in range(n):
        ct, tag = get("ct", i), get("tag", i)
        o = int(out_off[i])
        assert np.array_equal(out[o:o + ct.size], ct), i
        if tag.size >= TAG:
            assert np.array_equal(out[o + ct.size:o + ct.size + TAG], tag[:TAG]), i
            checked_tags += 1
    assert checked_tags >= 66
    # open what we sealed
    buf = np.concatenate([data[:int(ad_len.astype(np.int64).sum())], out])
    ct_off = out_off + np.uint64(int(ad_len.astype(np.int64).sum()))
    ct_len = (in_len.astype(np.uint64) + TAG).astype(np.uint16)
    dout_off = offsets(in_len)
    dec, ok = open_(ctx, keys, pre, kidx, pn, None, buf, ad_off, ad_len, ct_off, ct_len, dout_off,
                    int(in_len.astype(np.int64).sum()) + 1, host=host)
    assert ok.all()
    for i in range(n):
        o = int(dout_off[i])
        assert np.array_equal(dec[o:o + pts[i].size], pts[i]), i


def random_batch(n, seed, nkeys=5, lmax=1452):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 256, 32 * nkeys, dtype=np.uint8)
    pre = rng.integers(0, 256, 4 * nkeys, dtype=np.uint8)
    kidx = rng.integers(0, nkeys, n).astype(np.uint32)
    pn = rng.integers(1, 2**48, n, dtype=np.uint64)
    path = rng.integers(0, 3, n).astype(np.uint8)
    ad_len = rng.integers(0, 60, n).astype(np.uint16)
    in_len = rng.integers(0, lmax + 1, n).astype(np.uint16)
    gaps = rng.integers(0, 9, 2 * n).astype(np.uint64)
    lens = np.empty(2 * n, np.uint64)
    lens[0::2] = ad_len
    lens[1::2] = in_len
    off = offsets(lens + gaps) + gaps
    data = rng.integers(0, 256, int(off[-1] + lens[-1]) + 1, dtype=np.uint8)
    return keys, pre, kidx, pn, path, data, off[0::2].copy(), ad_len, off[1::2].copy(), in_len


@pytest.mark.parametrize("lmax", [15, 17, 64, 1452])
def test_seal_open_random_vs_oracle(ctx, lmax):
    n = 20_000 if lmax == 1452 else 3000
    keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len = random_batch(n, lmax, lmax=lmax)
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    size = int(in_len.astype(np.int64).sum()) + TAG * n
    got = seal(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size)
    want = OC.quic_c20p1305_encrypt_batch(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off,
                                          in_len, out_off, size, threads=8)
    assert np.array_equal(got, want)
    # open, every 4th packet tampered (ciphertext, tag or header)
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)] +
                         [np.zeros(1, np.uint8)])
    h_off = offsets(ad_len)
    ct = got.copy()
    ct_len = (in_len.astype(np.uint64) + TAG).astype(np.uint16)
    flip = np.arange(0, n, 4)
    pos = out_off[flip] + (np.arange(flip.size) * 7 % ct_len[flip].astype(np.uint64))
    ct[pos.astype(np.int64)] ^= 0x01
    buf = np.concatenate([hdr, ct])
    ct_off = out_off + np.uint64(hdr.size)
    d_off = offsets(in_len)
    dsize = int(in_len.astype(np.int64).sum()) + 1
    out, ok = open_(ctx, keys, pre, kidx, pn, path, buf, h_off, ad_len, ct_off, ct_len, d_off, dsize)
    w_out, w_ok = OC.quic_c20p1305_decrypt_batch(keys, pre, kidx, pn, path, buf, h_off, ad_len,
                                                 ct_off, ct_len, d_off, dsize)
    assert np.array_equal(ok, w_ok)
    assert w_ok[flip].sum() == 0 and w_ok.sum() == n - flip.size
    good = np.repeat(ok.astype(bool), in_len.astype(np.int64))
    assert np.array_equal(out[:good.size][good], w_out[:good.size][good])
    assert (out[:good.size][~good] == 0xA5).all()  # untouched on a bad tag


def test_seal_in_place(ctx):
    n = 4000
    keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len = random_batch(n, 77)
    rec = ad_len.astype(np.uint64) + in_len.astype(np.uint64) + TAG
    base = offsets(rec)
    buf = np.zeros(int(rec.sum()), np.uint8)
    a_off = base
    p_off = base + ad_len.astype(np.uint64)
    for p in range(n):
        buf[int(a_off[p]):int(a_off[p]) + int(ad_len[p])] = data[int(ad_off[p]):int(ad_off[p]) + int(ad_len[p])]
        buf[int(p_off[p]):int(p_off[p]) + int(in_len[p])] = data[int(in_off[p]):int(in_off[p]) + int(in_len[p])]
    d = dv(buf)
    ctx.chacha20poly1305_seal(dv(keys), dv(pre), dv(kidx), dv(pn), dv(path), d, dv(a_off),
                              dv(ad_len), dv(p_off), dv(in_len), n, d, dv(p_off))
    ctx.sync()
    torch.cuda.synchronize()
    res = d.cpu().numpy()
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    want = OC.quic_c20p1305_encrypt_batch(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off,
                                          in_len, out_off, int(out_off[-1]) + int(in_len[-1]) + TAG)
    for p in range(n):
        l_ = int(in_len[p]) + TAG
        assert np.array_equal(res[int(p_off[p]):int(p_off[p]) + l_],
                              want[int(out_off[p]):int(out_off[p]) + l_]), p
