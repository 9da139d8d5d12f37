"""CPU tests of the ChaCha20-Poly1305 oracle (oracle/qaead_oracle.c): pinned by
BoringSSL's own test vectors from the reference tree
(tests/golden/chacha20_poly1305.npz, made by tests/golden/make_golden_aead.py
from boringssl/crypto/cipher/test/chacha20_poly1305_tests.txt) and, for the
primitives, by the reference's chacha.c / poly1305_vec.c compiled into
oracle/_ref (skipped where that build is absent)."""
import numpy as np
import pytest

from oracle import oracle_c as OC
from oracle import ref_quic as R

from conftest import load_npz


@pytest.fixture(scope="module")
def vec():
    z = load_npz("chacha20_poly1305.npz")

    def get(f, i):
        o, l = int(z[f + "_off"][i]), int(z[f + "_len"][i])
        return z[f][o:o + l]
    return z, get


@pytest.fixture(scope="module")
def ref():
    if not R.available() and not R.build():
        pytest.skip("reference build oracle/_ref absent (no /root/reference here)")
    return R


def test_boringssl_vectors_seal_open(vec):
    z, get = vec
    n = z["key_len"].size
    assert n == 81
    for i in range(n):
        key, nonce, pt, ad, ct, tag = (get(f, i) for f in ("key", "nonce", "in", "ad", "ct", "tag"))
        out = OC.c20p1305_seal(key, nonce, pt, ad, tag_len=tag.size)
        assert np.array_equal(out[:pt.size], ct), i
        assert np.array_equal(out[pt.size:], tag), i
        ok, dec = OC.c20p1305_open(key, nonce, out, ad, tag_len=tag.size)
        assert ok and np.array_equal(dec, pt), i
        bad = out.copy()
        bad[-1] ^= 1
        assert not OC.c20p1305_open(key, nonce, bad, ad, tag_len=tag.size)[0], i


def test_rfc7539_keystream_kat():
    # RFC 7539 §2.4.2: key 00..1f, nonce 000000000000004a00000000, counter 1
    key = bytes(range(32))
    nonce = bytes.fromhex("000000000000004a00000000")
    pt = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip "
          b"for the future, sunscreen would be it.")
    ct = OC.chacha20(key, nonce, pt, counter=1)
    assert bytes(ct[:16]).hex() == "6e2e359a2568f98041ba0728dd0d6981"


def test_rfc7539_poly1305_kat():
    # RFC 7539 §2.5.2
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    tag = OC.poly1305(key, b"Cryptographic Forum Research Group")
    assert bytes(tag).hex() == "a8061dc1305136c6c22b8baf0c0127a9"


def test_primitives_vs_reference_random(ref):
    rng = np.random.default_rng(5)
    for _ in range(200):
        key = rng.integers(0, 256, 32, dtype=np.uint8)
        nonce = rng.integers(0, 256, 12, dtype=np.uint8)
        data = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8)
        ctr = int(rng.integers(0, 2**32 - 64))
        assert np.array_equal(OC.chacha20(key, nonce, data, ctr), ref.chacha20(key, nonce, data, ctr))
        split = int(rng.integers(0, data.size + 1))
        assert np.array_equal(OC.poly1305(key, data), ref.poly1305(key, data, split))


def test_quic_packet_form():
    rng = np.random.default_rng(9)
    key = rng.integers(0, 256, 32, dtype=np.uint8)
    prefix = rng.integers(0, 256, 4, dtype=np.uint8)
    ad = rng.integers(0, 256, 21, dtype=np.uint8)
    pt = rng.integers(0, 256, 1350, dtype=np.uint8)
    pn = 0x0000123456789ABC
    ct = OC.quic_c20p1305_encrypt(key, prefix, pn, ad, pt)
    # == RFC AEAD with nonce prefix || LE64(packet number), tag truncated to 12
    nonce = np.concatenate([prefix, np.frombuffer(pn.to_bytes(8, "little"), np.uint8)])
    assert np.array_equal(ct, OC.c20p1305_seal(key, nonce, pt, ad, tag_len=12))
    ok, back = OC.quic_c20p1305_decrypt(key, prefix, pn, ad, ct)
    assert ok and np.array_equal(back, pt)
    assert not OC.quic_c20p1305_decrypt(key, prefix, pn + 1, ad, ct)[0]
    # path id occupies the top byte of the packed packet number
    ct7 = OC.quic_c20p1305_encrypt(key, prefix, pn, ad, pt, path_id=7)
    nonce7 = np.concatenate([prefix, np.frombuffer(((7 << 56) | pn).to_bytes(8, "little"), np.uint8)])
    assert np.array_equal(ct7, OC.c20p1305_seal(key, nonce7, pt, ad, tag_len=12))


# ---- AES-128-GCM -------------------------------------------------------------
@pytest.fixture(scope="module")
def gvec():
    z = load_npz("aes_128_gcm.npz")

    def get(f, i):
        o, l = int(z[f + "_off"][i]), int(z[f + "_len"][i])
        return z[f][o:o + l]
    return z, get


def test_aes_fips197_kat():
    # FIPS-197 Appendix C.1
    key = bytes(range(16))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert bytes(OC.aes128_encrypt(key, pt)).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_boringssl_gcm_vectors(gvec):
    z, get = gvec
    n = z["key_len"].size
    assert n == 74
    for i in range(n):
        key, iv, pt, ad, ct, tag = (get(f, i) for f in ("key", "nonce", "in", "ad", "ct", "tag"))
        out = OC.aes128gcm_seal(key, iv, pt, ad, tag_len=tag.size)
        assert np.array_equal(out[:pt.size], ct), i
        assert np.array_equal(out[pt.size:], tag), i
        ok, dec = OC.aes128gcm_open(key, iv, out, ad, tag_len=tag.size)
        assert ok and np.array_equal(dec, pt), i
        bad = out.copy()
        bad[0 if out.size else 0] ^= 1
        if bad.size:
            assert not OC.aes128gcm_open(key, iv, bad, ad, tag_len=tag.size)[0], i


def test_gcm_vs_reference_random(ref):
    rng = np.random.default_rng(13)
    for _ in range(150):
        key = rng.integers(0, 256, 16, dtype=np.uint8)
        blk = rng.integers(0, 256, 16, dtype=np.uint8)
        assert np.array_equal(OC.aes128_encrypt(key, blk), ref.aes128_encrypt(key, blk))
        iv = rng.integers(0, 256, 12 if rng.integers(0, 4) else int(rng.integers(1, 40)),
                          dtype=np.uint8)
        pt = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8)
        ad = rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8)
        assert np.array_equal(OC.aes128gcm_seal(key, iv, pt, ad, 12),
                              ref.aes128gcm_seal(key, iv, pt, ad, 12))


def test_quic_gcm_batch_vs_reference(ref):
    """The QUIC packet form (prefix || LE64 packet number nonce, 12-byte tag,
    many keys) over the reference's gcm.c — the bench's CPU baseline — equals
    the oracle's batch."""
    rng = np.random.default_rng(17)
    n = 300
    L = rng.integers(0, 1453, n).astype(np.uint16)
    A = rng.integers(0, 40, n).astype(np.uint16)
    rec = A.astype(np.uint64) + L
    ad_off = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.uint64)
    pt_off = ad_off + A
    data = rng.integers(0, 256, int(rec.sum()), dtype=np.uint8)
    out_off = np.concatenate([[0], np.cumsum(L.astype(np.uint64) + 12)[:-1]]).astype(np.uint64)
    tot = int((L.astype(np.uint64) + 12).sum())
    keys = rng.integers(0, 256, 16 * 5, dtype=np.uint8)
    pre = rng.integers(0, 256, 4 * 5, dtype=np.uint8)
    kidx = rng.integers(0, 5, n).astype(np.uint32)
    pn = rng.integers(1, 2**40, n).astype(np.uint64)
    a = ref.quic_aes128gcm_encrypt_batch(keys, pre, kidx, pn, data, ad_off, A, pt_off, L,
                                         out_off, tot, threads=2)
    b = OC.quic_aes128gcm_encrypt_batch(keys, pre, kidx, pn, None, data, ad_off, A, pt_off, L,
                                        out_off, tot)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("aead", ["aes128gcm", "chacha20poly1305"])
def test_reference_asm_encrypters_match_oracle(aead):
    """The CPU baseline's library (oracle/_ref/libref_aead_asm.so: the
    reference's Aes128Gcm12Encrypter / ChaCha20Poly1305Encrypter over
    BoringSSL built WITH its x86-64 assembly) seals exactly what the oracle
    does — so the baseline times the same work — on multi-key batches of
    0..1452-byte payloads, on 1 and 4 threads."""
    if not R.asm_available():
        if not R.build() or not R.asm_available():
            pytest.skip("reference build oracle/_ref absent (no /root/reference here)")
    feats = R.asm_cpu_features()
    print(feats)
    rng = np.random.default_rng(11)
    n = 300
    ad_len = rng.integers(0, 40, n).astype(np.uint16)
    pt_len = rng.integers(0, 1453, n).astype(np.uint16)
    rec = ad_len.astype(np.uint64) + pt_len.astype(np.uint64)
    ad_off = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.uint64)
    pt_off = ad_off + ad_len.astype(np.uint64)
    data = rng.integers(0, 256, int(rec.sum()), dtype=np.uint8)
    out_len = pt_len.astype(np.uint64) + np.uint64(12)
    out_off = np.concatenate([[0], np.cumsum(out_len)[:-1]]).astype(np.uint64)
    kl = 16 if aead == "aes128gcm" else 32
    keys = rng.integers(0, 256, 5 * kl, dtype=np.uint8)
    pre = rng.integers(0, 256, 5 * 4, dtype=np.uint8)
    kidx = rng.integers(0, 5, n).astype(np.uint32)
    pn = rng.integers(1, 1 << 40, n).astype(np.uint64)
    size = int(out_len.sum())
    seal = OC.quic_aes128gcm_encrypt_batch if aead == "aes128gcm" else OC.quic_c20p1305_encrypt_batch
    want = seal(keys, pre, kidx, pn, None, data, ad_off, ad_len, pt_off, pt_len, out_off, size)
    for th in (1, 4):
        got = R.asm_seal_batch(aead, keys, pre, kidx, pn, data, ad_off, ad_len, pt_off, pt_len,
                               out_off, size, threads=th)
        assert np.array_equal(got, want), th
