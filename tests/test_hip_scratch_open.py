"""QFEC_SCRATCH_OUTPUT for the AEAD opens (ChaCha20-Poly1305, AES-128-GCM-12):
one pass over the ciphertext, MAC and decryption from the same slab loads.

Checked against the oracles (oracle/qaead_oracle.c, pinned by BoringSSL's
vectors — tests/test_oracle_aead.py): ok[] equal to the oracle's for random
multi-key batches with every 4th packet tampered (a ciphertext or tag byte);
verified packets' plaintext byte-exact; and a FAILED packet's output is its
unverified plaintext — keystream XOR the (tampered) ciphertext, i.e. the
original plaintext XOR the tamper — which is what BoringSSL's open leaves in
its output (it decrypts before it compares) and what QuicFramer's scratch
buffer tolerates (quic_framer.cc:1884-1930).  The default two-pass opens keep
the output untouched (tests/test_hip_aead.py, test_hip_gcm.py).
"""
import numpy as np
import pytest
import torch

from oracle import oracle_c as OC

from test_hip_aead import DEV, TAG, dv, offsets

pytestmark = pytest.mark.gpu


def _batch(n, seed, klen, nkeys, lmax):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 256, klen * nkeys, dtype=np.uint8)
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


@pytest.mark.parametrize("cipher", ["chacha20poly1305", "aes128gcm"])
@pytest.mark.parametrize("nkeys,lmax", [(1, 1452), (4, 1452), (2, 17)])
def test_open_scratch_output(ctx, cipher, nkeys, lmax):
    n = 12_000 if lmax > 64 else 3000
    klen = 32 if cipher == "chacha20poly1305" else 16
    enc = getattr(OC, f"quic_{'c20p1305' if klen == 32 else 'aes128gcm'}_encrypt_batch")
    dec = getattr(OC, f"quic_{'c20p1305' if klen == 32 else 'aes128gcm'}_decrypt_batch")
    keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len = _batch(
        n, 900 + nkeys + lmax + klen, klen, nkeys, lmax)
    out_off = offsets(in_len.astype(np.uint64) + TAG)
    size = int(in_len.astype(np.int64).sum()) + TAG * n
    ct0 = enc(keys, pre, kidx, pn, path, data, ad_off, ad_len, in_off, in_len, out_off, size,
              threads=8)
    hdr = np.concatenate([data[int(o):int(o) + int(l)] for o, l in zip(ad_off, ad_len)] +
                         [np.zeros(1, np.uint8)])
    h_off = offsets(ad_len)
    ct = ct0.copy()
    ct_len = (in_len.astype(np.uint64) + TAG).astype(np.uint16)
    flip = np.arange(0, n, 4)
    flip = flip[ct_len[flip] > 0]
    pos = out_off[flip] + (np.arange(flip.size) * 7 % ct_len[flip].astype(np.uint64))
    ct[pos.astype(np.int64)] ^= 0x01
    buf = np.concatenate([hdr, ct])
    ct_off = out_off + np.uint64(hdr.size)
    d_off = offsets(in_len) + np.uint64(3)
    dsize = int(in_len.astype(np.int64).sum()) + 4
    out = torch.full((dsize,), 0xA5, dtype=torch.uint8, device=DEV)
    ok = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    getattr(ctx, f"{cipher}_open")(dv(keys), dv(pre), dv(kidx), dv(pn), dv(path), dv(buf),
                                   dv(h_off), dv(ad_len), dv(ct_off), dv(ct_len), n, out,
                                   dv(d_off), ok, scratch_out=True)
    ctx.sync()
    torch.cuda.synchronize()
    out, ok = out.cpu().numpy(), ok.cpu().numpy()
    w_out, w_ok = dec(keys, pre, kidx, pn, path, buf, h_off, ad_len, ct_off, ct_len, d_off, dsize)
    assert np.array_equal(ok, w_ok)
    assert w_ok[flip].sum() == 0 and w_ok.sum() == n - flip.size
    # every packet's output: plaintext XOR the tamper of its ciphertext bytes
    # (zero for verified packets and for a tampered tag)
    for p in range(n):
        o, l = int(d_off[p]), int(in_len[p])
        c = int(out_off[p])
        pt = data[int(in_off[p]):int(in_off[p]) + l]
        want = pt ^ ct[c:c + l] ^ ct0[c:c + l]
        assert np.array_equal(out[o:o + l], want), (p, bool(ok[p]))
    good = np.repeat(ok.astype(bool), in_len.astype(np.int64))
    assert np.array_equal(out[3:3 + good.size][good], w_out[3:3 + good.size][good])
