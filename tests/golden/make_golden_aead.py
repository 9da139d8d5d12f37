"""Convert BoringSSL's ChaCha20-Poly1305 test vectors — data files in the
reference tree (/root/reference/boringssl/crypto/cipher/test/
chacha20_poly1305_tests.txt: RFC 7539 §2.8.2 and A.5 plus BoringSSL's own
cases, tags truncated to 1..16 bytes) — into tests/golden/chacha20_poly1305.npz.
Run in the container that has /root/reference:
    python tests/golden/make_golden_aead.py
"""
import os
import sys

import numpy as np

SRC = "/root/reference/boringssl/crypto/cipher/test/chacha20_poly1305_tests.txt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "chacha20_poly1305.npz")


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
    cases = parse(sys.argv[1] if len(sys.argv) > 1 else SRC)
    assert all(set(c) == {"KEY", "NONCE", "IN", "AD", "CT", "TAG"} for c in cases)
    d = {}
    for f in ("KEY", "NONCE", "IN", "AD", "CT", "TAG"):
        b, o, l = pack([c[f] for c in cases])
        d[f.lower()], d[f.lower() + "_off"], d[f.lower() + "_len"] = b, o, l
    np.savez_compressed(OUT, **d)
    print(f"{len(cases)} vectors -> {OUT}")


if __name__ == "__main__":
    main()
