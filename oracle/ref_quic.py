"""ctypes loader for oracle/_ref/libref_quic.so — the REFERENCE's own
NullEncrypter / NullDecrypter / QuicUtils::FNV1a_128_Hash_Two compiled from
/root/reference by oracle/ref/Makefile.

TEST INFRASTRUCTURE ONLY: used to pin oracle/qpp_oracle.c
(tests/test_oracle_protect.py) and to generate tests/golden/null_protect.npz.
Absent on a box without the reference build; callers skip then.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "_ref", "libref_quic.so")
REF = "/root/reference"
_lib = None


def build() -> bool:
    """Build from /root/reference when it exists (this container only)."""
    if os.path.isdir(REF):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(_HERE, "ref"), f"REF={REF}"], check=True)
    return os.path.exists(SO)


def available() -> bool:
    return os.path.exists(SO)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(SO)
        L.ref_fnv1a128_two.restype = None
        L.ref_fnv1a128_two.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        for fn in (L.ref_null_encrypt, L.ref_null_decrypt):
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                           C.c_size_t, C.POINTER(C.c_size_t)]
        L.ref_chacha20.restype = None
        L.ref_chacha20.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                   C.c_uint32]
        L.ref_poly1305.restype = None
        L.ref_poly1305.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.ref_aes128_encrypt.restype = None
        L.ref_aes128_encrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.ref_aes128gcm_seal.restype = C.c_int
        L.ref_aes128gcm_seal.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                         C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                         C.c_size_t]
        L.ref_null_encrypt_batch.restype = None
        L.ref_null_encrypt_batch.argtypes = [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p,
                                                                C.c_void_p, C.c_int]
        L.ref_quic_aes128gcm_seal_batch.restype = None
        L.ref_quic_aes128gcm_seal_batch.argtypes = [C.c_void_p] * 4 + [C.c_uint32] + \
            [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.ref_sent_entropy_run.restype = None
        L.ref_sent_entropy_run.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                           C.c_uint64] + [C.c_void_p] * 6
        _lib = L
    return _lib


def _b(x):
    a = np.frombuffer(bytes(x), dtype=np.uint8) if not isinstance(x, np.ndarray) else x
    return np.ascontiguousarray(a, dtype=np.uint8)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a.size else None


def fnv1a128_two(d1, d2=None):
    a = _b(d1)
    lo, hi = C.c_uint64(0), C.c_uint64(0)
    if d2 is None:
        lib().ref_fnv1a128_two(_ptr(a), a.size, None, 0, C.byref(lo), C.byref(hi))
    else:
        b = _b(d2)
        # a non-null pointer even for an empty second part (the reference
        # distinguishes nullptr, quic_utils.cc:121)
        pb = b.ctypes.data_as(C.c_void_p) if b.size else C.cast(C.create_string_buffer(1), C.c_void_p)
        lib().ref_fnv1a128_two(_ptr(a), a.size, pb, b.size, C.byref(lo), C.byref(hi))
    return int(hi.value) << 64 | int(lo.value)


def null_encrypt(ad, pt, cap=None):
    a, p = _b(ad), _b(pt)
    cap = p.size + 12 if cap is None else cap
    out = np.zeros(max(cap, 1), np.uint8)
    n = C.c_size_t(0)
    ok = lib().ref_null_encrypt(_ptr(a), a.size, _ptr(p), p.size, out.ctypes.data_as(C.c_void_p),
                                cap, C.byref(n))
    return bool(ok), out[:n.value].copy()


def null_decrypt(ad, ct, cap=None):
    a, c = _b(ad), _b(ct)
    cap = max(c.size - 12, 0) if cap is None else cap
    out = np.zeros(max(cap, 1), np.uint8)
    n = C.c_size_t(0)
    ok = lib().ref_null_decrypt(_ptr(a), a.size, _ptr(c), c.size, out.ctypes.data_as(C.c_void_p),
                                cap, C.byref(n))
    return bool(ok), out[:n.value].copy()


def chacha20(key, nonce, data, counter=0):
    """BoringSSL CRYPTO_chacha_20 (the reference's C implementation)."""
    k, n, d = _b(key), _b(nonce), _b(data)
    out = np.zeros(max(d.size, 1), np.uint8)
    lib().ref_chacha20(out.ctypes.data_as(C.c_void_p), _ptr(d), d.size, _ptr(k), _ptr(n), counter)
    return out[:d.size].copy()


def poly1305(key, msg, split=0):
    """BoringSSL CRYPTO_poly1305_{init,update,finish} (poly1305_vec.c)."""
    k, m = _b(key), _b(msg)
    tag = np.zeros(16, np.uint8)
    lib().ref_poly1305(tag.ctypes.data_as(C.c_void_p), _ptr(m), m.size, _ptr(k), split)
    return tag


def aes128_encrypt(key, block):
    """BoringSSL AES_set_encrypt_key + AES_encrypt (aes.c)."""
    k, b = _b(key), _b(block)
    out = np.zeros(16, np.uint8)
    lib().ref_aes128_encrypt(out.ctypes.data_as(C.c_void_p), _ptr(b), _ptr(k))
    return out


def aes128gcm_seal(key, iv, pt, ad, tag_len=16):
    """aead_aes_gcm_seal's sequence over BoringSSL's CRYPTO_gcm128_* (gcm.c)."""
    k, n, p, a = _b(key), _b(iv), _b(pt), _b(ad)
    out = np.zeros(p.size + tag_len, np.uint8)
    ok = lib().ref_aes128gcm_seal(out.ctypes.data_as(C.c_void_p), _ptr(k), _ptr(n), n.size, _ptr(p),
                                  p.size, _ptr(a), a.size, tag_len)
    assert ok
    return out


def _pa(a):
    return a.ctypes.data_as(C.c_void_p)


def null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, out_off, out_size, threads=1, out=None):
    """NullEncrypter::EncryptPacket per packet (CPU baseline, bench.py)."""
    out = np.zeros(out_size, np.uint8) if out is None else out
    lib().ref_null_encrypt_batch(_pa(data), _pa(ad_off), _pa(ad_len), _pa(pt_off), _pa(pt_len),
                                 pt_len.size, _pa(out), _pa(out_off), threads)
    return out


def quic_aes128gcm_encrypt_batch(keys, prefixes, key_idx, packet_number, data, ad_off, ad_len,
                                 pt_off, pt_len, out_off, out_size, threads=1, out=None):
    """Aes128Gcm12Encrypter-equivalent seal per packet over the reference's
    aes.c + gcm.c (CPU baseline, bench.py)."""
    out = np.zeros(out_size, np.uint8) if out is None else out
    n_keys = int(key_idx.max()) + 1 if key_idx.size else 0
    lib().ref_quic_aes128gcm_seal_batch(_pa(keys), _pa(prefixes), _pa(key_idx),
                                        _pa(packet_number), n_keys, _pa(data), _pa(ad_off),
                                        _pa(ad_len), _pa(pt_off), _pa(pt_len), pt_len.size,
                                        _pa(out), _pa(out_off), threads)
    return out


def sent_entropy_run(entropy, first_pn, largest, claimed, range_ptr, lo, hi):
    """QuicSentEntropyManager (quic_sent_entropy_manager.cc) of one connection:
    record packets 1..len(entropy), ClearEntropyBefore(first_pn),
    GetCumulativeEntropy(first_pn..), then IsValidEntropy per query."""
    e = np.ascontiguousarray(entropy, np.uint8)
    n = e.size
    cum = np.zeros(max(n - first_pn + 1, 1), np.uint8)
    ok = np.zeros(max(largest.size, 1), np.uint8)
    lib().ref_sent_entropy_run(_pa(e), n, first_pn, _pa(cum), largest.size, _pa(largest),
                               _pa(claimed), _pa(range_ptr), _pa(lo), _pa(hi), _pa(ok))
    return cum[:n - first_pn + 1], ok[:largest.size]


# ---- oracle/_ref/libref_aead_asm.so: the reference's encrypter classes over
# BoringSSL WITH its x86-64 assembly (oracle/ref/Makefile, ref_aead_shim.cc):
# the CPU speed the GPU protection kernels are compared with in bench.py.
ASM_SO = os.path.join(_HERE, "_ref", "libref_aead_asm.so")
_asm = None


def asm_available() -> bool:
    return os.path.exists(ASM_SO)


def asm_lib():
    global _asm
    if _asm is None:
        L = C.CDLL(ASM_SO)
        L.ref_aead_asm_seal_batch.restype = C.c_uint64
        L.ref_aead_asm_seal_batch.argtypes = [C.c_int] + [C.c_void_p] * 9 + \
            [C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.ref_aead_asm_ia32cap.restype = None
        L.ref_aead_asm_ia32cap.argtypes = [C.c_void_p]
        _asm = L
    return _asm


def asm_cpu_features() -> dict:
    """What BoringSSL detected (OPENSSL_ia32cap_P) and so which code it runs."""
    cap = (C.c_uint32 * 4)()
    asm_lib().ref_aead_asm_ia32cap(cap)
    return {"aesni": bool(cap[1] >> 25 & 1), "pclmulqdq": bool(cap[1] >> 1 & 1),
            "avx": bool(cap[1] >> 28 & 1), "avx2": bool(cap[2] >> 5 & 1),
            "ssse3": bool(cap[1] >> 9 & 1)}


def asm_seal_batch(aead, keys, prefixes, key_idx, packet_number, data, ad_off, ad_len, pt_off,
                   pt_len, out_off, out_size, threads=1, out=None):
    """Aes128Gcm12Encrypter (aead "aes128gcm") / ChaCha20Poly1305Encrypter
    ("chacha20poly1305") ::EncryptPacket per packet, BoringSSL assembly."""
    out = np.zeros(out_size, np.uint8) if out is None else out
    bad = asm_lib().ref_aead_asm_seal_batch(
        0 if aead == "aes128gcm" else 1, _pa(keys), _pa(prefixes), _pa(key_idx),
        _pa(packet_number), _pa(data), _pa(ad_off), _pa(ad_len), _pa(pt_off), _pa(pt_len),
        pt_len.size, _pa(out), _pa(out_off), threads)
    if bad:
        raise RuntimeError(f"reference EncryptPacket failed for {bad} packets")
    return out
