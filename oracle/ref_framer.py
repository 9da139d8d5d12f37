"""ctypes loader for oracle/_ref/libref_framer.so — the REFERENCE's QuicFramer
compiled from /root/reference by oracle/ref/Makefile (release build, no
stand-ins; C API in oracle/ref/ref_framer_shim.cc).

TEST INFRASTRUCTURE ONLY: the checker of the v<=31 FEC wire rows.  The
product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "_ref", "libref_framer.so")
_lib = None


class ParseResult(C.Structure):
    _fields_ = [("accepted", C.c_int32), ("error", C.c_int32), ("header_seen", C.c_int32),
                ("entropy_flag", C.c_int32), ("fec_flag", C.c_int32), ("n_ack", C.c_int32),
                ("n_ping", C.c_int32), ("n_padding", C.c_int32), ("n_stream", C.c_int32),
                ("complete", C.c_int32), ("packet_number", C.c_uint64),
                ("ack_largest_observed", C.c_uint64), ("ack_missing_count", C.c_uint64),
                ("detailed_error", C.c_char * 256)]


def available() -> bool:
    return os.path.exists(SO)


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(SO)
        L.ref_framer_parse.restype = C.c_int
        L.ref_framer_parse.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.POINTER(ParseResult)]
        L.ref_framer_public_header.restype = C.c_size_t
        L.ref_framer_public_header.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_void_p,
                                               C.c_size_t]
        L.ref_framer_build.restype = C.c_size_t
        L.ref_framer_build.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                       C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t,
                                       C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.ref_framer_encrypt.restype = C.c_size_t
        L.ref_framer_encrypt.argtypes = [C.c_int, C.c_uint64, C.c_void_p, C.c_size_t,
                                         C.c_size_t, C.c_size_t]
        _lib = L
    return _lib


def parse(version: int, packet: bytes) -> dict:
    r = ParseResult()
    buf = (C.c_uint8 * max(1, len(packet))).from_buffer_copy(packet or b"\0")
    lib().ref_framer_parse(version, C.addressof(buf), len(packet), C.byref(r))
    d = {f: getattr(r, f) for f, _ in ParseResult._fields_}
    d["detailed_error"] = r.detailed_error.decode()
    return d


def public_header(version: int, packet_number: int, pn_len: int) -> bytes:
    buf = (C.c_uint8 * 64)()
    n = lib().ref_framer_public_header(version, packet_number, pn_len, C.addressof(buf), 64)
    assert n, "AppendPacketHeader failed"
    return bytes(buf[:n])


def build(version: int, packet_number: int, pn_len: int, entropy: bool, kind: str,
          largest_observed: int = 0, missing=()):
    """(plaintext packet, associated-data length) from QuicFramer::BuildDataPacket;
    kind "ack" (missing: [(lo, hi), ...] half-open) or "ping"."""
    lo = (C.c_uint64 * max(1, len(missing)))(*[m[0] for m in missing])
    hi = (C.c_uint64 * max(1, len(missing)))(*[m[1] for m in missing])
    buf = (C.c_uint8 * 1452)()
    ad = C.c_size_t(0)
    n = lib().ref_framer_build(version, packet_number, pn_len, int(entropy),
                               0 if kind == "ack" else 1, largest_observed, C.addressof(lo),
                               C.addressof(hi), len(missing), C.addressof(buf), 1452, C.byref(ad))
    assert n, "BuildDataPacket failed"
    return bytes(buf[:n]), ad.value


def encrypt(version: int, packet_number: int, plaintext: bytes, ad_len: int) -> bytes:
    """NullEncrypter over plaintext[ad_len:] (QuicFramer::EncryptInPlace)."""
    cap = len(plaintext) + 12
    buf = (C.c_uint8 * cap).from_buffer_copy(plaintext + b"\0" * 12)
    n = lib().ref_framer_encrypt(version, packet_number, C.addressof(buf), ad_len,
                                 len(plaintext), cap)
    assert n, "EncryptInPlace failed"
    return bytes(buf[:n])
