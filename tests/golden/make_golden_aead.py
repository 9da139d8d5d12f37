"""Convert BoringSSL's AEAD test vectors — data files in the reference tree
(/root/reference/boringssl/crypto/cipher/test/chacha20_poly1305_tests.txt:
RFC 7539 §2.8.2 and A.5 plus BoringSSL's own cases, tags truncated to 1..16
bytes; aes_128_gcm_tests.txt: the GCM spec / NIST cases, 8..64-byte IVs) —
into tests/golden/{chacha20_poly1305,aes_128_gcm}.npz.
Run in the container that has /root/reference:
    python tests/golden/make_golden_aead.py
"""
import os
import sys

import numpy as np

TESTS = "/root/reference/boringssl/crypto/cipher/test/"
HERE = os.path.dirname(os.path.abspath(__file__))
FILES = {"chacha20_poly1305_tests.txt": "chacha20_poly1305.npz",
         "aes_128_gcm_tests.txt": "aes_128_gcm.npz"}


def value(v):
    v = v.strip()
    if v.startswith('"'):
        return v[1:-1].encode()
    return bytes.fromhex(v)


def parse(path):
    cases, cur = [], {}
    for line in open(path):
        line = line.rstrip("\n")
        if not line.strip() or line.startswith("#"):
            if cur:
                cases.append(cur)
                cur = {}
            continue
        k, v = line.split(":", 1)
        cur[k.strip()] = value(v)
    if cur:
        cases.append(cur)
    return cases


def pack(vals):
    off = np.zeros(len(vals), np.uint64)
    ln = np.array([len(v) for v in vals], np.uint32)
    off[1:] = np.cumsum(ln.astype(np.uint64))[:-1]
    return np.frombuffer(b"".join(vals), np.uint8).copy(), off, ln


def main():
    for src, dst in FILES.items():
        cases = parse(os.path.join(TESTS, src))
        assert all(set(c) == {"KEY", "NONCE", "IN", "AD", "CT", "TAG"} for c in cases)
        d = {}
        for f in ("KEY", "NONCE", "IN", "AD", "CT", "TAG"):
            b, o, l = pack([c[f] for c in cases])
            d[f.lower()], d[f.lower() + "_off"], d[f.lower() + "_len"] = b, o, l
        out = os.path.join(HERE, dst)
        np.savez_compressed(out, **d)
        print(f"{len(cases)} vectors -> {out}")


if __name__ == "__main__":
    main()
