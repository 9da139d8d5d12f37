"""Generate tests/golden/null_protect.npz from the REFERENCE's own
NullEncrypter / NullDecrypter (oracle/_ref/libref_quic.so, built from
/root/reference by oracle/ref/Makefile).  Run in the container that has
/root/reference:  python tests/golden/make_golden_protect.py

Layout (CSR, one shared byte buffer):
  data            all inputs: per packet its header (associated data) then payload
  ad_off, ad_len  header of packet p
  pt_off, pt_len  plaintext of packet p
  ct              concatenated reference ciphertexts (12-byte tag || plaintext)
  ct_off, ct_len  ciphertext of packet p inside ct
  dec_*           decrypt cases: ciphertexts (some tampered / truncated) with the
                  reference's verdict dec_ok and plaintext output dec_pt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ref_quic as R  # noqa: E402


def main():
    assert R.build(), "reference build failed (needs /root/reference)"
    rng = np.random.default_rng(0x4E554C4C)
    pt_lens = [0, 1, 2, 7, 8, 11, 12, 13, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 256,
               1000, 1337, 1338, 1339, 1350, 1440, 1451, 1452]
    pt_lens += list(rng.integers(0, 1453, 36))
    ad_lens = [0, 1, 9, 10, 13, 16, 17, 19, 22, 28, 41] + list(rng.integers(0, 52, len(pt_lens) - 11))
    data, ad_off, ad_len, pt_off, pt_len = [], [], [], [], []
    ct, ct_off, ct_len = [], [], []
    pos = cpos = 0
    for a_n, p_n in zip(ad_lens, pt_lens):
        ad = rng.integers(0, 256, int(a_n), dtype=np.uint8)
        pt = rng.integers(0, 256, int(p_n), dtype=np.uint8)
        ok, c = R.null_encrypt(ad, pt)
        assert ok and c.size == pt.size + 12
        data += [ad, pt]
        ad_off.append(pos); ad_len.append(ad.size); pos += ad.size
        pt_off.append(pos); pt_len.append(pt.size); pos += pt.size
        ct.append(c); ct_off.append(cpos); ct_len.append(c.size); cpos += c.size
    data = np.concatenate(data).astype(np.uint8)
    ctb = np.concatenate(ct).astype(np.uint8)
    # decrypt cases: every ciphertext as is, plus tampered tag / payload /
    # header, truncated below the tag, and the empty ciphertext
    dec_data, dec_ad_off, dec_ad_len, dec_ct_off, dec_ct_len, dec_ok, dec_pt = [], [], [], [], [], [], []
    dpos = 0
    for p in range(len(pt_len)):
        ad = data[ad_off[p]:ad_off[p] + ad_len[p]].copy()
        c = ctb[ct_off[p]:ct_off[p] + ct_len[p]].copy()
        variants = [(ad, c)]
        if p % 3 == 0:
            t = c.copy(); t[p % 12] ^= 0x01; variants.append((ad, t))
        if p % 3 == 1 and c.size > 12:
            t = c.copy(); t[12 + (p * 7) % (c.size - 12)] ^= 0x80; variants.append((ad, t))
        if p % 3 == 2 and ad.size:
            a2 = ad.copy(); a2[-1] ^= 0x10; variants.append((a2, c))
        if p % 11 == 0:
            variants.append((ad, c[:p % 12]))
        for a_, c_ in variants:
            ok, out = R.null_decrypt(a_, c_)
            dec_data += [a_, c_]
            dec_ad_off.append(dpos); dec_ad_len.append(a_.size); dpos += a_.size
            dec_ct_off.append(dpos); dec_ct_len.append(c_.size); dpos += c_.size
            dec_ok.append(int(ok))
            dec_pt.append(out if ok else np.zeros(0, np.uint8))
    kat = np.array([R.fnv1a128_two(b"") & ((1 << 64) - 1), R.fnv1a128_two(b"") >> 64],
                   dtype=np.uint64)
    np.savez_compressed(
        os.path.join(os.path.dirname(os.path.abspath(__file__)), "null_protect.npz"),
        data=data, ad_off=np.array(ad_off, np.uint64), ad_len=np.array(ad_len, np.uint16),
        pt_off=np.array(pt_off, np.uint64), pt_len=np.array(pt_len, np.uint16),
        ct=ctb, ct_off=np.array(ct_off, np.uint64), ct_len=np.array(ct_len, np.uint16),
        dec_data=np.concatenate(dec_data).astype(np.uint8),
        dec_ad_off=np.array(dec_ad_off, np.uint64), dec_ad_len=np.array(dec_ad_len, np.uint16),
        dec_ct_off=np.array(dec_ct_off, np.uint64), dec_ct_len=np.array(dec_ct_len, np.uint16),
        dec_ok=np.array(dec_ok, np.uint8),
        dec_pt=np.concatenate(dec_pt).astype(np.uint8) if dec_pt else np.zeros(0, np.uint8),
        fnv_empty=kat)
    print(f"{len(pt_len)} encrypt cases, {len(dec_ok)} decrypt cases "
          f"({sum(dec_ok)} valid), {data.size + ctb.size} bytes")


if __name__ == "__main__":
    main()
