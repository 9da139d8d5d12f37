"""ctypes loader for the C oracle (oracle/build/libqfec_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by libquic_amd/.  See qfec_oracle.h for
the contract and the "parity unpinned" status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libqfec_oracle.so")
_lib = None

u8p = C.POINTER(C.c_uint8)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        L.qo_entropy_cumulative_batch.restype = None
        L.qo_entropy_cumulative_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                                  C.c_void_p]
        L.qo_entropy_validate_batch.restype = None
        L.qo_entropy_validate_batch.argtypes = [C.c_void_p] * 10 + [C.c_uint64, C.c_void_p]
        L.qo_packet_entropy_hash.restype = C.c_uint8
        L.qo_packet_entropy_hash.argtypes = [C.c_int, C.c_uint64]
        L.qo_splitmix64.restype = C.c_uint64
        L.qo_splitmix64.argtypes = [C.c_uint64]
        L.qo_synth_fixed.restype = None
        L.qo_synth_fixed.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                     C.c_uint64, C.c_uint64, C.c_void_p]
        L.qo_synth_row.restype = None
        L.qo_synth_row.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
        L.qo_ragged_k.restype = C.c_uint32
        L.qo_ragged_k.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]
        L.qo_ragged_len.restype = C.c_uint32
        L.qo_ragged_len.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.qo_drop_index.restype = C.c_uint32
        L.qo_drop_index.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.qo_encode_fixed.restype = C.c_int
        L.qo_encode_fixed.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64,
                                      C.c_uint64, C.c_void_p, C.c_uint64]
        L.qo_recover_fixed.restype = C.c_int
        L.qo_recover_fixed.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                       C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p,
                                       C.c_uint64]
        L.qo_encode_ragged.restype = C.c_int
        L.qo_encode_ragged.argtypes = [C.c_void_p] * 4 + [C.c_uint64] + [C.c_void_p] * 3
        L.qo_recover_ragged.restype = C.c_int
        L.qo_recover_ragged.argtypes = [C.c_void_p] * 4 + [C.c_uint64] + [C.c_void_p] * 6
        L.qo_encode_fixed_mt.restype = C.c_int
        L.qo_encode_fixed_mt.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64,
                                         C.c_void_p, C.c_int]
        L.qo_recover_fixed_mt.restype = C.c_int
        L.qo_recover_fixed_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                          C.c_uint32, C.c_uint64, C.c_void_p, C.c_int]
        L.qo_fnv1a64.restype = C.c_uint64
        L.qo_fnv1a64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.qo_time_single_group_ns.restype = C.c_double
        L.qo_time_single_group_ns.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        L.qo_group_digest.restype = C.c_uint64
        L.qo_group_digest.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p,
                                      C.c_void_p, C.c_int]
        L.qo_ragged_digests.restype = None
        L.qo_ragged_digests.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.qo_fixed_digests.restype = None
        L.qo_fixed_digests.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                       C.c_uint32, C.c_int, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]
        # packet protection (qpp_oracle.h)
        L.qo_fnv1a128_two.restype = None
        L.qo_fnv1a128_two.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        for fn in (L.qo_null_encrypt, L.qo_null_decrypt):
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                           C.c_size_t, C.POINTER(C.c_size_t)]
        L.qo_null_encrypt_batch.restype = None
        L.qo_null_encrypt_batch.argtypes = [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p,
                                                               C.c_void_p]
        L.qo_null_decrypt_batch.restype = None
        L.qo_null_decrypt_batch.argtypes = [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p,
                                                               C.c_void_p, C.c_void_p]
        L.qo_null_encrypt_batch_mt.restype = None
        L.qo_null_encrypt_batch_mt.argtypes = [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p,
                                                                  C.c_void_p, C.c_int]
        # ChaCha20-Poly1305 (qaead_oracle.h)
        L.qo_chacha20.restype = None
        L.qo_chacha20.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                  C.c_uint32]
        L.qo_poly1305.restype = None
        L.qo_poly1305.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        for fn in (L.qo_c20p1305_seal, L.qo_c20p1305_open):
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                           C.c_void_p, C.c_size_t, C.c_size_t]
        for fn in (L.qo_quic_c20p1305_encrypt, L.qo_quic_c20p1305_decrypt):
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint8, C.c_uint64,
                           C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.qo_quic_c20p1305_encrypt_batch.restype = None
        L.qo_quic_c20p1305_encrypt_batch.argtypes = [C.c_void_p] * 10 + [C.c_uint64, C.c_void_p,
                                                                        C.c_void_p, C.c_int]
        L.qo_quic_c20p1305_decrypt_batch.restype = None
        L.qo_quic_c20p1305_decrypt_batch.argtypes = [C.c_void_p] * 10 + [C.c_uint64, C.c_void_p,
                                                                        C.c_void_p, C.c_void_p]
        # AES-128-GCM
        L.qo_aes128_expand.restype = None
        L.qo_aes128_expand.argtypes = [C.c_void_p, C.c_void_p]
        L.qo_aes128_encrypt.restype = None
        L.qo_aes128_encrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        for fn in (L.qo_aes128gcm_seal, L.qo_aes128gcm_open):
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                           C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t]
        L.qo_quic_aes128gcm_encrypt_batch.restype = None
        L.qo_quic_aes128gcm_encrypt_batch.argtypes = [C.c_void_p] * 10 + [
            C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.qo_quic_aes128gcm_decrypt_batch.restype = None
        L.qo_quic_aes128gcm_decrypt_batch.argtypes = [C.c_void_p] * 10 + [
            C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def synth_fixed(seed, g0, n, k, L, row_stride=None, group_stride=None):
    rs = L if row_stride is None else row_stride
    gs = k * rs if group_stride is None else group_stride
    rows = np.zeros(n * gs, dtype=np.uint8)
    lib().qo_synth_fixed(seed, g0, n, k, L, rs, gs, _p(rows))
    return rows


def encode_fixed(rows, k, L, n, row_stride=None, group_stride=None, parity_stride=None):
    rs = L if row_stride is None else row_stride
    gs = k * rs if group_stride is None else group_stride
    ps = L if parity_stride is None else parity_stride
    par = np.zeros(n * ps, dtype=np.uint8)
    rc = lib().qo_encode_fixed(_p(rows), k, L, rs, gs, n, _p(par), ps)
    return rc, par


def recover_fixed(rows, parity, missing, k, L, n, row_stride=None, group_stride=None,
                  parity_stride=None, out_stride=None):
    rs = L if row_stride is None else row_stride
    gs = k * rs if group_stride is None else group_stride
    ps = L if parity_stride is None else parity_stride
    os_ = L if out_stride is None else out_stride
    out = np.zeros(n * os_, dtype=np.uint8)
    missing = np.ascontiguousarray(missing, dtype=np.uint8)
    rc = lib().qo_recover_fixed(_p(rows), _p(parity), _p(missing), k, L, rs, gs, ps, n,
                                _p(out), os_)
    return rc, out


def encode_ragged(data, pkt_off, pkt_len, grp_ptr, parity_off, parity_size):
    n = grp_ptr.size - 1
    par = np.zeros(parity_size, dtype=np.uint8)
    plen = np.zeros(n, dtype=np.uint16)
    rc = lib().qo_encode_ragged(_p(data), _p(pkt_off), _p(pkt_len), _p(grp_ptr), n, _p(par),
                                _p(parity_off), _p(plen))
    return rc, par, plen


def recover_ragged(data, pkt_off, pkt_len, grp_ptr, parity, parity_off, parity_len, missing,
                   out_off, out_size):
    n = grp_ptr.size - 1
    out = np.zeros(out_size, dtype=np.uint8)
    missing = np.ascontiguousarray(missing, dtype=np.uint8)
    rc = lib().qo_recover_ragged(_p(data), _p(pkt_off), _p(pkt_len), _p(grp_ptr), n, _p(parity),
                                 _p(parity_off), _p(parity_len), _p(missing), _p(out),
                                 _p(out_off))
    return rc, out


def fnv1a64(buf: np.ndarray, h: int = 0) -> int:
    buf = np.ascontiguousarray(buf)
    return int(lib().qo_fnv1a64(_p(buf), buf.nbytes, h))


def group_digest(base, n, stride=0, L=0, off=None, lens=None, threads=None):
    """Checksum of per-group checksums (see qfec_oracle.h)."""
    threads = threads or min(16, os.cpu_count() or 1)
    return int(lib().qo_group_digest(_p(base), n, stride, L,
                                     None if off is None else _p(off),
                                     None if lens is None else _p(lens), threads))


def fixed_digests(seed, drop_seed, g0, n, k, L, threads=None):
    threads = threads or min(16, os.cpu_count() or 1)
    a, b = C.c_uint64(0), C.c_uint64(0)
    lib().qo_fixed_digests(seed, drop_seed, g0, n, k, L, threads, C.byref(a), C.byref(b))
    return int(a.value), int(b.value)


def ragged_digests(seed, drop_seed, g0, n, kmin=5, kmax=15, lmin=64, lmax=1350, threads=None):
    threads = threads or min(16, os.cpu_count() or 1)
    a, b = C.c_uint64(0), C.c_uint64(0)
    lib().qo_ragged_digests(seed, drop_seed, g0, n, kmin, kmax, lmin, lmax, threads, C.byref(a),
                            C.byref(b))
    return int(a.value), int(b.value)


# ---- packet protection (qpp_oracle.h) -------------------------------------
NULL_TAG = 12  # kHashSizeShort, null_encrypter.cc:15


def _buf(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
    return np.ascontiguousarray(a, dtype=np.uint8)


def fnv1a128_two(d1, d2=None):
    a = _buf(d1)
    lo, hi = C.c_uint64(0), C.c_uint64(0)
    if d2 is None:
        lib().qo_fnv1a128_two(_p(a), a.size, None, 0, C.byref(lo), C.byref(hi))
    else:
        b = _buf(d2)
        lib().qo_fnv1a128_two(_p(a), a.size, _p(b), b.size, C.byref(lo), C.byref(hi))
    return int(hi.value) << 64 | int(lo.value)


def null_encrypt(ad, pt):
    a, p = _buf(ad), _buf(pt)
    out = np.zeros(p.size + NULL_TAG, np.uint8)
    n = C.c_size_t(0)
    ok = lib().qo_null_encrypt(_p(a), a.size, _p(p), p.size, _p(out), out.size, C.byref(n))
    return bool(ok), out[:n.value]


def null_decrypt(ad, ct):
    a, c = _buf(ad), _buf(ct)
    out = np.zeros(max(c.size - NULL_TAG, 0) + 1, np.uint8)
    n = C.c_size_t(0)
    ok = lib().qo_null_decrypt(_p(a), a.size, _p(c), c.size, _p(out), out.size, C.byref(n))
    return bool(ok), out[:n.value]


def null_encrypt_batch(data, ad_off, ad_len, pt_off, pt_len, out_off, out_size, threads=1, out=None):
    out = np.zeros(out_size, np.uint8) if out is None else out
    args = [_p(data), _p(ad_off), _p(ad_len), _p(pt_off), _p(pt_len), pt_len.size, _p(out),
            _p(out_off)]
    if threads > 1:
        lib().qo_null_encrypt_batch_mt(*args, threads)
    else:
        lib().qo_null_encrypt_batch(*args)
    return out


def null_decrypt_batch(data, ad_off, ad_len, ct_off, ct_len, out_off, out_size):
    out = np.zeros(out_size, np.uint8)
    ok = np.zeros(ct_len.size, np.uint8)
    lib().qo_null_decrypt_batch(_p(data), _p(ad_off), _p(ad_len), _p(ct_off), _p(ct_len),
                                ct_len.size, _p(out), _p(out_off), _p(ok))
    return out, ok


# ---- ChaCha20-Poly1305 (qaead_oracle.h) -----------------------------------
AEAD_TAG = 12  # kAuthTagSize, chacha20_poly1305_encrypter.h


def _pn(a):
    return _p(a) if a.size else None


def chacha20(key, nonce, data, counter=0):
    k, n, d = _buf(key), _buf(nonce), _buf(data)
    out = np.zeros(max(d.size, 1), np.uint8)
    lib().qo_chacha20(_p(out), _pn(d), d.size, _p(k), _p(n), counter)
    return out[:d.size]


def poly1305(key, msg):
    k, m = _buf(key), _buf(msg)
    tag = np.zeros(16, np.uint8)
    lib().qo_poly1305(_p(tag), _pn(m), m.size, _p(k))
    return tag


def c20p1305_seal(key, nonce, pt, ad, tag_len=16):
    k, n, p, a = _buf(key), _buf(nonce), _buf(pt), _buf(ad)
    out = np.zeros(p.size + tag_len, np.uint8)
    lib().qo_c20p1305_seal(_p(out), _p(k), _p(n), _pn(p), p.size, _pn(a), a.size, tag_len)
    return out


def c20p1305_open(key, nonce, ct, ad, tag_len=16):
    k, n, c, a = _buf(key), _buf(nonce), _buf(ct), _buf(ad)
    out = np.zeros(max(c.size - tag_len, 0) + 1, np.uint8)
    ok = lib().qo_c20p1305_open(_p(out), _p(k), _p(n), _pn(c), c.size, _pn(a), a.size, tag_len)
    return bool(ok), out[:max(c.size - tag_len, 0)]


def quic_c20p1305_encrypt(key, prefix, packet_number, ad, pt, path_id=0):
    k, x, a, p = _buf(key), _buf(prefix), _buf(ad), _buf(pt)
    out = np.zeros(p.size + AEAD_TAG, np.uint8)
    lib().qo_quic_c20p1305_encrypt(_p(out), _p(k), _p(x), path_id, packet_number, _pn(a), a.size,
                                   _pn(p), p.size)
    return out


def quic_c20p1305_decrypt(key, prefix, packet_number, ad, ct, path_id=0):
    k, x, a, c = _buf(key), _buf(prefix), _buf(ad), _buf(ct)
    out = np.zeros(max(c.size - AEAD_TAG, 0) + 1, np.uint8)
    ok = lib().qo_quic_c20p1305_decrypt(_p(out), _p(k), _p(x), path_id, packet_number, _pn(a),
                                        a.size, _pn(c), c.size)
    return bool(ok), out[:max(c.size - AEAD_TAG, 0)]


def quic_c20p1305_encrypt_batch(keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                                ad_len, pt_off, pt_len, out_off, out_size, threads=1, out=None):
    out = np.zeros(out_size, np.uint8) if out is None else out
    lib().qo_quic_c20p1305_encrypt_batch(
        _p(keys), _p(prefixes), _p(key_idx), _p(packet_number),
        None if path_id is None else _p(path_id), _p(data), _p(ad_off), _p(ad_len), _p(pt_off),
        _p(pt_len), pt_len.size, _p(out), _p(out_off), threads)
    return out


def quic_c20p1305_decrypt_batch(keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                                ad_len, ct_off, ct_len, out_off, out_size):
    out = np.zeros(out_size, np.uint8)
    ok = np.zeros(ct_len.size, np.uint8)
    lib().qo_quic_c20p1305_decrypt_batch(
        _p(keys), _p(prefixes), _p(key_idx), _p(packet_number),
        None if path_id is None else _p(path_id), _p(data), _p(ad_off), _p(ad_len), _p(ct_off),
        _p(ct_len), ct_len.size, _p(out), _p(out_off), _p(ok))
    return out, ok


# ---- AES-128-GCM (qaead_oracle.h) ------------------------------------------
def aes128_encrypt(key, block):
    k, b = _buf(key), _buf(block)
    rk = np.zeros(44, np.uint32)
    lib().qo_aes128_expand(_p(rk), _p(k))
    out = np.zeros(16, np.uint8)
    lib().qo_aes128_encrypt(_p(out), _p(b), _p(rk))
    return out


def aes128gcm_seal(key, iv, pt, ad, tag_len=16):
    k, n, p, a = _buf(key), _buf(iv), _buf(pt), _buf(ad)
    out = np.zeros(p.size + tag_len, np.uint8)
    lib().qo_aes128gcm_seal(_p(out), _p(k), _p(n), n.size, _pn(p), p.size, _pn(a), a.size, tag_len)
    return out


def aes128gcm_open(key, iv, ct, ad, tag_len=16):
    k, n, c, a = _buf(key), _buf(iv), _buf(ct), _buf(ad)
    out = np.zeros(max(c.size - tag_len, 0) + 1, np.uint8)
    ok = lib().qo_aes128gcm_open(_p(out), _p(k), _p(n), n.size, _pn(c), c.size, _pn(a), a.size,
                                 tag_len)
    return bool(ok), out[:max(c.size - tag_len, 0)]


def quic_aes128gcm_encrypt_batch(keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                                 ad_len, pt_off, pt_len, out_off, out_size, threads=1, out=None):
    out = np.zeros(out_size, np.uint8) if out is None else out
    lib().qo_quic_aes128gcm_encrypt_batch(
        _p(keys), _p(prefixes), _p(key_idx), _p(packet_number),
        None if path_id is None else _p(path_id), _p(data), _p(ad_off), _p(ad_len), _p(pt_off),
        _p(pt_len), pt_len.size, _p(out), _p(out_off), threads)
    return out


def quic_aes128gcm_decrypt_batch(keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                                 ad_len, ct_off, ct_len, out_off, out_size):
    out = np.zeros(out_size, np.uint8)
    ok = np.zeros(ct_len.size, np.uint8)
    lib().qo_quic_aes128gcm_decrypt_batch(
        _p(keys), _p(prefixes), _p(key_idx), _p(packet_number),
        None if path_id is None else _p(path_id), _p(data), _p(ad_off), _p(ad_len), _p(ct_off),
        _p(ct_len), ct_len.size, _p(out), _p(out_off), _p(ok))
    return out, ok


# ---- entropy bookkeeping (qent_oracle.c) ------------------------------------
def packet_entropy_hash(flag, packet_number):
    return int(lib().qo_packet_entropy_hash(int(bool(flag)), int(packet_number)))


def entropy_cumulative_batch(entropy, conn_ptr, cum_base):
    cum = np.zeros(entropy.size, np.uint8)
    n = conn_ptr.size - 1
    lib().qo_entropy_cumulative_batch(_p(entropy), _p(conn_ptr),
                                      None if cum_base is None else _p(cum_base), n, _p(cum))
    return cum


def entropy_validate_batch(cum, conn_ptr, first_pn, cum_base, ack_conn, largest, claimed,
                           range_ptr, range_lo, range_hi):
    ok = np.zeros(ack_conn.size, np.uint8)
    lib().qo_entropy_validate_batch(_p(cum), _p(conn_ptr), _p(first_pn),
                                    None if cum_base is None else _p(cum_base), _p(ack_conn),
                                    _p(largest), _p(claimed), _p(range_ptr), _p(range_lo),
                                    _p(range_hi), ack_conn.size, _p(ok))
    return ok
