"""CPU tests of the packet-protection oracle (oracle/qpp_oracle.c): pinned
against the REFERENCE's own NullEncrypter / NullDecrypter / FNV1a_128_Hash_Two
(oracle/_ref/libref_quic.so, built from /root/reference — skipped where that
build is absent) and against the fixtures that build generated
(tests/golden/null_protect.npz, always)."""
import numpy as np
import pytest

from oracle import oracle_c as OC
from oracle import ref_quic as R

from conftest import load_npz

FNV128_OFFSET = 144066263297769815596495629667062367629  # quic_utils.cc:114-116 (published FNV basis)


@pytest.fixture(scope="module")
def gold():
    return load_npz("null_protect.npz")


@pytest.fixture(scope="module")
def ref():
    if not R.available() and not R.build():
        pytest.skip("reference build oracle/_ref absent (no /root/reference here)")
    return R


def test_fnv_offset_basis_kat(gold):
    assert OC.fnv1a128_two(b"") == FNV128_OFFSET
    assert int(gold["fnv_empty"][1]) << 64 | int(gold["fnv_empty"][0]) == FNV128_OFFSET


def test_encrypt_matches_reference_fixtures(gold):
    g = gold
    for p in range(g["pt_len"].size):
        ad = g["data"][int(g["ad_off"][p]):int(g["ad_off"][p]) + int(g["ad_len"][p])]
        pt = g["data"][int(g["pt_off"][p]):int(g["pt_off"][p]) + int(g["pt_len"][p])]
        ok, ct = OC.null_encrypt(ad, pt)
        want = g["ct"][int(g["ct_off"][p]):int(g["ct_off"][p]) + int(g["ct_len"][p])]
        assert ok and np.array_equal(ct, want), p


def test_decrypt_matches_reference_fixtures(gold):
    g = gold
    pos = 0
    for p in range(g["dec_ok"].size):
        ad = g["dec_data"][int(g["dec_ad_off"][p]):int(g["dec_ad_off"][p]) + int(g["dec_ad_len"][p])]
        ct = g["dec_data"][int(g["dec_ct_off"][p]):int(g["dec_ct_off"][p]) + int(g["dec_ct_len"][p])]
        ok, pt = OC.null_decrypt(ad, ct)
        assert ok == bool(g["dec_ok"][p]), p
        if ok:
            assert np.array_equal(pt, g["dec_pt"][pos:pos + pt.size]), p
            pos += pt.size
    assert pos == g["dec_pt"].size


def test_batch_forms_match_single(gold):
    g = gold
    out_off = np.zeros(g["pt_len"].size, np.uint64)
    out_off[1:] = np.cumsum(g["pt_len"].astype(np.uint64) + 12)[:-1]
    size = int(g["pt_len"].astype(np.int64).sum() + 12 * g["pt_len"].size)
    out = OC.null_encrypt_batch(g["data"], g["ad_off"], g["ad_len"], g["pt_off"], g["pt_len"],
                                out_off, size)
    assert np.array_equal(out, g["ct"])
    out4 = OC.null_encrypt_batch(g["data"], g["ad_off"], g["ad_len"], g["pt_off"], g["pt_len"],
                                 out_off, size, threads=4)
    assert np.array_equal(out4, g["ct"])
    dlen = np.maximum(g["dec_ct_len"].astype(np.int64) - 12, 0)
    doff = np.zeros(dlen.size, np.uint64)
    doff[1:] = np.cumsum(dlen)[:-1]
    dout, ok = OC.null_decrypt_batch(g["dec_data"], g["dec_ad_off"], g["dec_ad_len"],
                                     g["dec_ct_off"], g["dec_ct_len"], doff, int(dlen.sum()) + 1)
    assert np.array_equal(ok, g["dec_ok"])


def test_restatement_vs_reference_random(ref):
    rng = np.random.default_rng(7)
    for _ in range(300):
        ad = rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8)
        pt = rng.integers(0, 256, int(rng.integers(0, 1453)), dtype=np.uint8)
        assert OC.fnv1a128_two(ad, pt) == ref.fnv1a128_two(ad, pt)
        ok1, c1 = OC.null_encrypt(ad, pt)
        ok2, c2 = ref.null_encrypt(ad, pt)
        assert ok1 and ok2 and np.array_equal(c1, c2)
        t = c1.copy()
        if rng.integers(0, 2):
            t[int(rng.integers(0, t.size))] ^= 1 << int(rng.integers(0, 8))
        ok1, p1 = OC.null_decrypt(ad, t)
        ok2, p2 = ref.null_decrypt(ad, t)
        assert ok1 == ok2 and np.array_equal(p1, p2)


def test_reference_capacity_and_short_input(ref):
    # cap too small -> false in both (null_encrypter.cc:36-38, null_decrypter.cc:53-56)
    ok, _ = ref.null_encrypt(b"h", b"payload", cap=18)
    assert not ok
    assert not OC.null_decrypt(b"h", b"short")[0] and not ref.null_decrypt(b"h", b"short")[0]


def test_reference_batch_equals_oracle_batch(ref):
    """ref_null_encrypt_batch (the bench's reference CPU baseline) equals the
    oracle's batch on ragged packets."""
    rng = np.random.default_rng(23)
    n = 400
    L = rng.integers(0, 1453, n).astype(np.uint16)
    A = rng.integers(0, 40, n).astype(np.uint16)
    rec = A.astype(np.uint64) + L
    ad_off = np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.uint64)
    pt_off = ad_off + A
    data = rng.integers(0, 256, int(rec.sum()), dtype=np.uint8)
    out_off = np.concatenate([[0], np.cumsum(L.astype(np.uint64) + 12)[:-1]]).astype(np.uint64)
    tot = int((L.astype(np.uint64) + 12).sum())
    a = ref.null_encrypt_batch(data, ad_off, A, pt_off, L, out_off, tot, threads=2)
    b = OC.null_encrypt_batch(data, ad_off, A, pt_off, L, out_off, tot)
    assert np.array_equal(a, b)
