"""GPU parity tests of the AES-128-GCM packet-protection kernel (qpp_kernels.hip)
through the C-ABI (qfec_aes128gcm_seal/open_batch): BoringSSL's own GCM vectors
from the reference tree (the 69 with 96-bit nonces — QUIC's; ciphertext + the
12-byte tag prefix) and random batches against the vector- and
reference-pinned C oracle, for waves that share one key (4-bit GHASH table
path) and waves that mix keys (bit-serial GHASH path).  Bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC

from conftest import load_npz
from test_hip_aead import DEV, TAG, dv, offsets

pytestmark = pytest.mark.gpu


def seal(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size,
         host=False):
    n = in_len.size
    if host:
        out = np.zeros(size, np.uint8)
        ctx.aes128gcm_seal(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, n,
                           out, out_off, host=True)
        return out
    out = torch.zeros(size, dtype=torch.uint8, device=DEV)
    ctx.aes128gcm_seal(dv(keys), dv(pre), dv(kidx), dv(pn), None if path is None else dv(path),
                       dv(data), dv(ad_off), dv(ad_len), dv(in_off), dv(in_len), n, out,
                       dv(out_off))
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy()


def open_(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size,
          host=False, fill=0xA5):
    n = in_len.size
    if host:
        out = np.full(size, fill, np.uint8)
        ok = np.full(n, 7, np.uint8)
        ctx.aes128gcm_open(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, n,
                           out, out_off, ok, host=True)
        return out, ok
    out = torch.full((size,), fill, dtype=torch.uint8, device=DEV)
    ok = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    ctx.aes128gcm_open(dv(keys), dv(pre), dv(kidx), dv(pn), None if path is None else dv(path),
                       dv(data), dv(ad_off), dv(ad_len), dv(in_off), dv(in_len), n, out,
                       dv(out_off), ok)
    ctx.sync()
    torch.cuda.synchronize()
    return out.cpu().numpy(), ok.cpu().numpy()


@pytest.mark.parametrize("host", [False, True])
def test_boringssl_gcm_vectors(ctx, host):
    z = load_npz("aes_128_gcm.npz")

    def get(f, i):
        o, l = int(z[f + "_off"][i]), int(z[f + "_len"][i])
        return z[f][o:o + l]
    idx = [i for i in range(z["key_len"].size) if int(z["nonce_len"][i]) == 12]
    assert len(idx) == 69
    n = len(idx)
    keys = np.concatenate([get("key", i) for i in idx])
    nonces = [get("nonce", i) for i in idx]
    pre = np.concatenate([x[:4] for x in nonces])
    pn = np.array([int.from_bytes(bytes(x[4:]), "little") for x in nonces], np.uint64)
    kidx = np.arange(n, dtype=np.uint32)
    ads = [get("ad", i) for i in idx]
    pts = [get("in", i) for i in idx]
    ad_len = np.array([a.size for a in ads], np.uint16)
    in_len = np.array([p.size for p in pts], np.uint16)
    nad = int(ad_len.astype(np.int64).sum())
    data = np.concatenate(ads + pts + [np.zeros(1, np.uint8)])
    ad_off = offsets(ad_len)
    in_off = offsets(in_len) + np.uint64(nad)
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    size = int(in_len.astype(np.int64).sum()) + TAG * n
    out = seal(ctx, keys, pre, kidx, pn, None, data, ad_off, ad_len, in_off, in_len, out_off, size,
               host=host)
    for j, i in enumerate(idx):
        ct, tag = get("ct", i), get("tag", i)
        o = int(out_off[j])
        assert np.array_equal(out[o:o + ct.size], ct), i
        assert np.array_equal(out[o + ct.size:o + ct.size + TAG], tag[:TAG]), i
    buf = np.concatenate([data[:nad], out])
    ct_off = out_off + np.uint64(nad)
    ct_len = (in_len.astype(np.uint64) + TAG).astype(np.uint16)
    d_off = offsets(in_len)
    dec, ok = open_(ctx, keys, pre, kidx, pn, None, buf, ad_off, ad_len, ct_off, ct_len, d_off,
                    int(in_len.astype(np.int64).sum()) + 1, host=host)
    assert ok.all()
    for j in range(n):
        o = int(d_off[j])
        assert np.array_equal(dec[o:o + pts[j].size], pts[j]), j


def random_batch(n, seed, nkeys, lmax=1452):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 256, 16 * nkeys, dtype=np.uint8)
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


@pytest.mark.parametrize("nkeys,lmax", [(1, 1452), (5, 1452), (1, 17), (3, 15)])
def test_seal_open_random_vs_oracle(ctx, nkeys, lmax):
    n = 6000 if lmax == 1452 else 2000
    if nkeys > 1 and lmax == 1452:
        n = 1500  # mixed-key waves take the bit-serial GHASH
    keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len = random_batch(
        n, 100 + nkeys + lmax, nkeys, lmax)
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    size = int(in_len.astype(np.int64).sum()) + TAG * n
    got = seal(ctx, keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size)
    want = OC.quic_aes128gcm_encrypt_batch(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off,
                                           in_len, out_off, size, threads=8)
    assert np.array_equal(got, want)
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)] +
                         [np.zeros(1, np.uint8)])
    h_off = offsets(ad_len)
    ct = got.copy()
    ct_len = (in_len.astype(np.uint64) + TAG).astype(np.uint16)
    flip = np.arange(0, n, 4)
    pos = out_off[flip] + (np.arange(flip.size) * 7 % ct_len[flip].astype(np.uint64))
    ct[pos.astype(np.int64)] ^= 0x02
    buf = np.concatenate([hdr, ct])
    ct_off = out_off + np.uint64(hdr.size)
    d_off = offsets(in_len)
    dsize = int(in_len.astype(np.int64).sum()) + 1
    out, ok = open_(ctx, keys, pre, kidx, pn, path, buf, h_off, ad_len, ct_off, ct_len, d_off, dsize)
    w_out, w_ok = OC.quic_aes128gcm_decrypt_batch(keys, pre, kidx, pn, path, buf, h_off, ad_len,
                                                  ct_off, ct_len, d_off, dsize)
    assert np.array_equal(ok, w_ok)
    assert w_ok[flip].sum() == 0 and w_ok.sum() == n - flip.size
    good = np.repeat(ok.astype(bool), in_len.astype(np.int64))
    assert np.array_equal(out[:good.size][good], w_out[:good.size][good])
    assert (out[:good.size][~good] == 0xA5).all()



def test_block_shapes_agree_on_large_batch(ctx):
    """launch_aes128gcm seals batches of >= 2^22 packets with the 768-thread
    shape and smaller ones with the 512-thread shape: the same 2^22 packets
    sealed in one call and in two halves (in place, [header | payload | 12
    spare] records) must give the same bytes, and the (512-thread) open must
    verify every one of them.  Device-side compare."""
    n = 1 << 22
    rng = np.random.default_rng(41)
    hdr = 13
    pt_len = rng.integers(0, 81, n).astype(np.uint16)
    rec = hdr + pt_len.astype(np.uint64) + TAG
    ad_off = offsets(rec)
    in_off = ad_off + np.uint64(hdr)
    ad_len = np.full(n, hdr, np.uint16)
    total = int(ad_off[-1] + rec[-1])
    nkeys = 5
    keys = rng.integers(0, 256, 16 * nkeys, dtype=np.uint8)
    pre = rng.integers(0, 256, 4 * nkeys, dtype=np.uint8)
    kidx = (np.arange(n, dtype=np.uint32) // 192) % nkeys  # mostly key-uniform waves
    pn = np.arange(1, n + 1, dtype=np.uint64)
    d = {k: dv(v) for k, v in dict(ad_off=ad_off, ad_len=ad_len, in_off=in_off, in_len=pt_len,
                                     keys=keys, pre=pre, kidx=kidx, pn=pn).items()}
    base = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    whole, halves = base.clone(), base.clone()
    torch.cuda.synchronize()  # the context may run on a stream of its own
    ctx.aes128gcm_seal(d["keys"], d["pre"], d["kidx"], d["pn"], None, whole, d["ad_off"],
                       d["ad_len"], d["in_off"], d["in_len"], n, whole, d["in_off"])
    h = n // 2
    for lo in (0, h):
        sl = slice(lo, lo + h)
        ctx.aes128gcm_seal(d["keys"], d["pre"], d["kidx"][sl], d["pn"][sl], None, halves,
                           d["ad_off"][sl], d["ad_len"][sl], d["in_off"][sl], d["in_len"][sl], h,
                           halves, d["in_off"][sl])
    ctx.sync()
    torch.cuda.synchronize()
    assert torch.equal(whole, halves)
    ok = torch.zeros(n, dtype=torch.uint8, device=DEV)
    pout = torch.zeros(int(pt_len.astype(np.int64).sum()) + 1, dtype=torch.uint8, device=DEV)
    ctx.aes128gcm_open(d["keys"], d["pre"], d["kidx"], d["pn"], None, whole, d["ad_off"],
                       d["ad_len"], d["in_off"], dv((pt_len.astype(np.uint32) + TAG).astype(np.uint16)),
                       n, pout, dv(offsets(pt_len.astype(np.uint64))), ok)
    ctx.sync()
    torch.cuda.synchronize()
    assert bool(ok.all())
