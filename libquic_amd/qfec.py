"""ctypes binding of the qfec C-ABI (include/qfec.h) — test / bench plumbing.

The product is the native library ``libquic_amd/libqfec.so`` (HIP kernels +
C-ABI + the C++ QuicFecGroup host mirror).  This module only forwards calls;
it never computes FEC bytes itself and has no CPU fallback: if the library or
the GPU is missing, every call raises.

Buffers may be torch tensors (device or pinned host) or numpy arrays (host);
the caller picks ``host=True`` for host pointers (QFEC_PTR_HOST), or
``mapped=True`` for payloads in pinned host memory the kernels read in place
(QFEC_PTR_MAPPED; torch ``pin_memory()`` tensors or ``HostBuffer``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libqfec.so")

QFEC_OK = 0
QFEC_ERR_INTERNAL = -1
QFEC_ERR_INVALID_FEC_DATA = -5
QFEC_PTR_DEVICE = 0
QFEC_PTR_HOST = 1
QFEC_CACHED = 2
QFEC_PTR_MAPPED = 4
QFEC_ONE_PASS = 8
QFEC_ASYNC = 16
QFEC_SCRATCH_OUTPUT = 32
QFEC_SMALL_GROUPS = 64
QFEC_PENDING = 1
MAX_PACKET_SIZE = 1452
DEFAULT_MAX_PACKET_SIZE = 1350
MAX_GROUP_PACKETS = 255

# Every symbol include/qfec.h declares: (name, restype, argtypes)
_vp, _u8p = C.c_void_p, C.c_void_p
SIGNATURES = [
    ("qfec_abi_version", C.c_int, []),
    ("qfec_create", C.c_void_p, [C.c_int]),
    ("qfec_destroy", None, [C.c_void_p]),
    ("qfec_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("qfec_get_stream", C.c_void_p, [C.c_void_p]),
    ("qfec_own_stream", C.c_void_p, [C.c_void_p]),
    ("qfec_sync", C.c_int, [C.c_void_p]),
    ("qfec_strerror", C.c_char_p, [C.c_int]),
    ("qfec_last_error", C.c_char_p, [C.c_void_p]),
    ("qfec_host_alloc", C.c_void_p, [C.c_size_t]),
    ("qfec_host_free", None, [C.c_void_p]),
    ("qfec_host_register", C.c_int, [C.c_void_p, C.c_size_t]),
    ("qfec_host_unregister", C.c_int, [C.c_void_p]),
    ("qfec_encode_batch", C.c_int,
     [_vp, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, _u8p, C.c_uint32]),
    ("qfec_recover_batch", C.c_int,
     [_vp, _u8p, _u8p, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, _u8p, C.c_uint32]),
    ("qfec_encode_batch_strided", C.c_int,
     [_vp, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, _u8p, C.c_uint64,
      C.c_uint32]),
    ("qfec_recover_batch_strided", C.c_int,
     [_vp, _u8p, _u8p, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
      C.c_uint64, _u8p, C.c_uint64, C.c_uint32]),
    ("qfec_recover_inslot_batch", C.c_int,
     [_vp, _u8p, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, _u8p, C.c_uint32]),
    ("qfec_recover_inslot_batch_strided", C.c_int,
     [_vp, _u8p, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, _u8p,
      C.c_uint64, C.c_uint32]),
    ("qfec_encode_ragged", C.c_int,
     [_vp, _u8p, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, _vp, C.c_uint32]),
    ("qfec_recover_ragged", C.c_int,
     [_vp, _u8p, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, _vp, _u8p, _u8p, _vp, C.c_uint32]),
    ("qfec_xor_into", C.c_int, [_vp, _u8p, C.c_uint64, _u8p, C.c_uint32]),
    ("qfec_wire_write_private_header", C.c_size_t, [_vp, _u8p, C.c_size_t]),
    ("qfec_wire_parse_private_header", C.c_size_t,
     [_u8p, C.c_size_t, C.c_int, C.c_uint64, _vp]),
    ("qfec_wire_write_revived", C.c_size_t, [_vp, C.c_size_t, C.c_size_t, _u8p, C.c_size_t]),
    ("qfec_wire_parse_revived", C.c_size_t, [_u8p, C.c_size_t, C.c_size_t, _vp, _vp]),
    ("qfec_wire_fec_packet_body", C.c_size_t,
     [C.c_uint64, C.c_uint64, C.c_int, _u8p, C.c_size_t, _u8p, C.c_size_t]),
    ("qfec_null_encrypt_batch", C.c_int,
     [_vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, C.c_uint32]),
    ("qfec_null_decrypt_batch", C.c_int,
     [_vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, _u8p, C.c_uint32]),
    ("qfec_chacha20poly1305_seal_batch", C.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, C.c_uint32]),
    ("qfec_chacha20poly1305_open_batch", C.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, _u8p,
      C.c_uint32]),
    ("qfec_aes128gcm_seal_batch", C.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, C.c_uint32]),
    ("qfec_aes128gcm_open_batch", C.c_int,
     [_vp, _vp, _vp, _vp, _vp, _vp, _u8p, _vp, _vp, _vp, _vp, C.c_uint64, _u8p, _vp, _u8p,
      C.c_uint32]),
    ("qfec_entropy_cumulative_batch", C.c_int,
     [_vp, _u8p, _vp, _u8p, C.c_uint64, C.c_uint64, _u8p, C.c_uint32]),
    ("qfec_entropy_validate_batch", C.c_int,
     [_vp, _u8p, _vp, _vp, _u8p, C.c_uint64, _vp, _vp, _u8p, _vp, _vp, _vp, C.c_uint64, _u8p,
      C.c_uint32]),
    ("qfec_stream_probe", C.c_int, [_vp, _u8p, C.c_uint64, _u8p, C.c_int]),
    ("qfec_phase_abandons", C.c_int, [_vp, _vp]),
    ("qfec_phase_backoff", C.c_int, [_vp]),
    ("qfec_debug_phase", C.c_int, [_vp, C.c_uint32, C.c_int]),
    ("qfec_debug_phase_min", C.c_int, [_vp, C.c_uint32]),
    ("qfec_debug_phase_regsteps", C.c_int, [_vp, C.c_int]),
    ("qfec_debug_phase_rtbatch", C.c_int, [_vp, C.c_uint32]),
    ("qfec_debug_phase_reserve", C.c_int, [_vp, C.c_uint32]),
    ("qfec_debug_other_service_cus", C.c_uint32, [_vp, C.POINTER(C.c_uint32)]),
    ("qfec_last_fixed_phased", C.c_int, [_vp]),
    ("qfec_debug_last_phase_grid", C.c_uint32, [_vp]),
    ("qfec_debug_fail_launches", C.c_int, [_vp, C.c_int]),
    ("qfec_debug_service", C.c_int, [_vp, C.c_int, C.POINTER(C.c_uint64)]),
    ("qfec_debug_service_stamps", C.c_int, [_vp, C.c_int, C.POINTER(C.c_uint64)]),
    ("qfec_debug_service_trace", C.c_int, [_vp, C.POINTER(C.c_uint64)]),
    ("qfec_debug_service_feed", C.c_int, [_vp, C.c_int, C.POINTER(C.c_uint64)]),
    ("qfec_debug_service_resident", C.c_uint64, [_vp, C.c_uint64]),
    ("qfec_debug_service_idle", C.c_uint64, [_vp, C.c_uint64]),
    ("qfec_debug_service_hold", C.c_int, [_vp, C.c_int]),
    ("qfec_complete", C.c_int, [_vp, C.c_int]),
    ("qfec_async_ticket", C.c_uint64, [_vp]),
    ("qfec_complete_ticket", C.c_int, [_vp, C.c_uint64, C.c_int]),
    ("qfec_service_warm", C.c_int, [_vp]),
    ("qfec_synth_fixed", C.c_int,
     [_vp, _u8p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
      C.c_uint64]),
    ("qfec_synth_ragged", C.c_int,
     [_vp, _u8p, _vp, _vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64]),
]

_lib = None


class QfecError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


class InvalidFecData(QfecError):
    pass


def load(path: str = LIB_PATH):
    """Load libqfec.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise ImportError(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (the HIP path has no CPU fallback)")
        lib = C.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _fl(host=False, mapped=False, cached=False, one_pass=False):
    return ((QFEC_PTR_HOST if host else 0) | (QFEC_PTR_MAPPED if mapped else 0)
            | (QFEC_CACHED if cached else 0) | (QFEC_ONE_PASS if one_pass else 0))


class HostBuffer:
    """n bytes of pinned, device-mapped host memory from qfec_host_alloc, as a
    numpy uint8 view (.array); freed with close()."""

    def __init__(self, n: int):
        import numpy as np
        self.lib = load()
        self.ptr = self.lib.qfec_host_alloc(n)
        if not self.ptr:
            raise QfecError(QFEC_ERR_INTERNAL, self.lib.qfec_last_error(None).decode())
        self.n = n
        self.array = np.ctypeslib.as_array((C.c_uint8 * n).from_address(self.ptr))

    def close(self):
        if self.ptr:
            self.array = None
            self.lib.qfec_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostRegistration:
    """Pins and device-maps an existing host buffer (a numpy array, a CPU torch
    tensor or a raw address + size) for mapped=True calls; unregister() (or the
    end of a with-block) releases it.  The buffer must outlive the
    registration."""

    def __init__(self, buf, nbytes=None):
        self.lib = load()
        self.ptr = _ptr(buf)
        self.n = int(nbytes if nbytes is not None else
                     (buf.nbytes if hasattr(buf, "nbytes") else buf.numel() * buf.element_size()))
        rc = self.lib.qfec_host_register(self.ptr, self.n)
        if rc != QFEC_OK:
            raise QfecError(rc, self.lib.qfec_last_error(None).decode())

    def unregister(self):
        if self.ptr:
            rc = self.lib.qfec_host_unregister(self.ptr)
            self.ptr = None
            if rc != QFEC_OK:
                raise QfecError(rc, self.lib.qfec_last_error(None).decode())

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.unregister()


def _ptr(x):
    """Address of a torch tensor / numpy array / int / None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        assert x.flags["C_CONTIGUOUS"], "numpy buffers must be C-contiguous"
        return x.ctypes.data
    raise TypeError(f"unsupported buffer {type(x)!r}")


class Context:
    """One qfec_ctx (one device, one stream).  Thread-compatible, not thread-safe."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.ctx = self.lib.qfec_create(device)
        if not self.ctx:
            raise QfecError(QFEC_ERR_INTERNAL, self.lib.qfec_last_error(None).decode())
        self.device = device

    def close(self):
        if self.ctx:
            self.lib.qfec_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing --------------------------------------------------------
    def _check(self, rc: int):
        if rc != QFEC_OK:
            msg = self.lib.qfec_last_error(self.ctx).decode()
            if rc == QFEC_ERR_INVALID_FEC_DATA:
                raise InvalidFecData(rc, msg)
            raise QfecError(rc, msg)
        return rc

    def set_stream(self, stream):
        """stream: torch.cuda.Stream (its handle; torch's default stream is HIP's
        null stream, handle 0) / raw hipStream_t int / None (the context's own
        non-blocking stream)."""
        if stream is None:
            h = self.lib.qfec_own_stream(self.ctx)
        else:
            h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        return self._check(self.lib.qfec_set_stream(self.ctx, h or None))

    def sync(self):
        return self._check(self.lib.qfec_sync(self.ctx))

    # -- fixed -------------------------------------------------------------
    def encode(self, rows, k, L, n_groups, parity_out, *, row_stride=None, group_stride=None,
               parity_stride=None, host=False, cached=False, mapped=False, one_pass=False):
        fl = _fl(host, mapped, cached, one_pass)
        if row_stride is None and group_stride is None and parity_stride is None:
            rc = self.lib.qfec_encode_batch(self.ctx, _ptr(rows), k, L, n_groups,
                                            _ptr(parity_out), fl)
        else:
            rs = L if row_stride is None else row_stride
            gs = k * rs if group_stride is None else group_stride
            ps = L if parity_stride is None else parity_stride
            rc = self.lib.qfec_encode_batch_strided(self.ctx, _ptr(rows), k, L, rs, gs, n_groups,
                                                    _ptr(parity_out), ps, fl)
        return self._check(rc)

    def recover(self, rows, parity, missing, k, L, n_groups, out, *, row_stride=None,
                group_stride=None, parity_stride=None, out_stride=None, host=False,
                cached=False, mapped=False, one_pass=False):
        fl = _fl(host, mapped, cached, one_pass)
        if row_stride is None and group_stride is None and parity_stride is None \
                and out_stride is None:
            rc = self.lib.qfec_recover_batch(self.ctx, _ptr(rows), _ptr(parity), _ptr(missing),
                                             k, L, n_groups, _ptr(out), fl)
        else:
            rs = L if row_stride is None else row_stride
            gs = k * rs if group_stride is None else group_stride
            ps = L if parity_stride is None else parity_stride
            os_ = L if out_stride is None else out_stride
            rc = self.lib.qfec_recover_batch_strided(self.ctx, _ptr(rows), _ptr(parity),
                                                     _ptr(missing), k, L, rs, gs, ps, n_groups,
                                                     _ptr(out), os_, fl)
        return self._check(rc)

    def recover_inslot(self, rows, missing, k, L, n_groups, out=None, *, row_stride=None,
                       group_stride=None, out_stride=None, host=False, cached=False,
                       mapped=False, one_pass=False):
        """In-slot recover: rows[g][missing[g]] holds the redundancy; out=None
        writes the lost packet in place there (device pointers only)."""
        fl = _fl(host, mapped, cached, one_pass)
        if row_stride is None and group_stride is None and out_stride is None:
            rc = self.lib.qfec_recover_inslot_batch(self.ctx, _ptr(rows), _ptr(missing), k, L,
                                                    n_groups, _ptr(out), fl)
        else:
            rs = L if row_stride is None else row_stride
            gs = k * rs if group_stride is None else group_stride
            os_ = L if out_stride is None else out_stride
            rc = self.lib.qfec_recover_inslot_batch_strided(self.ctx, _ptr(rows), _ptr(missing),
                                                            k, L, rs, gs, n_groups, _ptr(out),
                                                            os_, fl)
        return self._check(rc)

    # -- ragged ------------------------------------------------------------
    def encode_ragged(self, data, pkt_off, pkt_len, grp_ptr, n_groups, parity_out, parity_off,
                      parity_len_out, *, host=False, mapped=False, async_=False,
                      small_groups=False):
        rc = self.lib.qfec_encode_ragged(self.ctx, _ptr(data), _ptr(pkt_off), _ptr(pkt_len),
                                         _ptr(grp_ptr), n_groups, _ptr(parity_out),
                                         _ptr(parity_off), _ptr(parity_len_out),
                                         _fl(host, mapped) | (QFEC_ASYNC if async_ else 0)
                                         | (QFEC_SMALL_GROUPS if small_groups else 0))
        return self._check(rc)

    def recover_ragged(self, data, pkt_off, pkt_len, grp_ptr, n_groups, parity, parity_off,
                       parity_len, missing, out, out_off, *, host=False, mapped=False,
                       async_=False, small_groups=False):
        rc = self.lib.qfec_recover_ragged(self.ctx, _ptr(data), _ptr(pkt_off), _ptr(pkt_len),
                                          _ptr(grp_ptr), n_groups, _ptr(parity),
                                          _ptr(parity_off), _ptr(parity_len), _ptr(missing),
                                          _ptr(out), _ptr(out_off),
                                          _fl(host, mapped) | (QFEC_ASYNC if async_ else 0)
                                          | (QFEC_SMALL_GROUPS if small_groups else 0))
        return self._check(rc)

    def xor_into(self, src, n, dst, *, host=False, mapped=False):
        return self._check(self.lib.qfec_xor_into(self.ctx, _ptr(src), n, _ptr(dst),
                                                  _fl(host, mapped)))

    # -- packet protection (ENCRYPTION_NONE) --------------------------------
    def null_encrypt(self, data, ad_off, ad_len, in_off, in_len, n, out, out_off, *, host=False):
        return self._check(self.lib.qfec_null_encrypt_batch(
            self.ctx, _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), QFEC_PTR_HOST if host else 0))

    def null_decrypt(self, data, ad_off, ad_len, in_off, in_len, n, out, out_off, ok, *,
                     host=False, scratch_out=False):
        """scratch_out: QFEC_SCRATCH_OUTPUT (one pass; a failed packet's output
        holds its unverified plaintext)."""
        fl = (QFEC_PTR_HOST if host else 0) | (QFEC_SCRATCH_OUTPUT if scratch_out else 0)
        return self._check(self.lib.qfec_null_decrypt_batch(
            self.ctx, _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), _ptr(ok), fl))

    def chacha20poly1305_seal(self, keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                              ad_len, in_off, in_len, n, out, out_off, *, host=False):
        return self._check(self.lib.qfec_chacha20poly1305_seal_batch(
            self.ctx, _ptr(keys), _ptr(prefixes), _ptr(key_idx), _ptr(packet_number),
            _ptr(path_id), _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), QFEC_PTR_HOST if host else 0))

    def chacha20poly1305_open(self, keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                              ad_len, in_off, in_len, n, out, out_off, ok, *, host=False,
                              scratch_out=False):
        fl = (QFEC_PTR_HOST if host else 0) | (QFEC_SCRATCH_OUTPUT if scratch_out else 0)
        return self._check(self.lib.qfec_chacha20poly1305_open_batch(
            self.ctx, _ptr(keys), _ptr(prefixes), _ptr(key_idx), _ptr(packet_number),
            _ptr(path_id), _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), _ptr(ok), fl))

    def aes128gcm_seal(self, keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                       ad_len, in_off, in_len, n, out, out_off, *, host=False):
        return self._check(self.lib.qfec_aes128gcm_seal_batch(
            self.ctx, _ptr(keys), _ptr(prefixes), _ptr(key_idx), _ptr(packet_number),
            _ptr(path_id), _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), QFEC_PTR_HOST if host else 0))

    def aes128gcm_open(self, keys, prefixes, key_idx, packet_number, path_id, data, ad_off,
                       ad_len, in_off, in_len, n, out, out_off, ok, *, host=False,
                       scratch_out=False):
        fl = (QFEC_PTR_HOST if host else 0) | (QFEC_SCRATCH_OUTPUT if scratch_out else 0)
        return self._check(self.lib.qfec_aes128gcm_open_batch(
            self.ctx, _ptr(keys), _ptr(prefixes), _ptr(key_idx), _ptr(packet_number),
            _ptr(path_id), _ptr(data), _ptr(ad_off), _ptr(ad_len), _ptr(in_off), _ptr(in_len), n,
            _ptr(out), _ptr(out_off), _ptr(ok), fl))

    # -- packet-entropy bookkeeping --------------------------------------------
    def entropy_cumulative(self, entropy, conn_ptr, cum_base, n_conns, cum, *, n_packets=0,
                           host=False):
        return self._check(self.lib.qfec_entropy_cumulative_batch(
            self.ctx, _ptr(entropy), _ptr(conn_ptr), _ptr(cum_base), n_conns, n_packets,
            _ptr(cum), QFEC_PTR_HOST if host else 0))

    def entropy_validate(self, cum, conn_ptr, first_pn, cum_base, n_conns, ack_conn, largest,
                         claimed, range_ptr, range_lo, range_hi, n_acks, ok, *, host=False):
        return self._check(self.lib.qfec_entropy_validate_batch(
            self.ctx, _ptr(cum), _ptr(conn_ptr), _ptr(first_pn), _ptr(cum_base), n_conns,
            _ptr(ack_conn), _ptr(largest), _ptr(claimed), _ptr(range_ptr), _ptr(range_lo),
            _ptr(range_hi), n_acks, _ptr(ok), QFEC_PTR_HOST if host else 0))

    def stream_probe(self, src, n, dst, copy=False):
        return self._check(self.lib.qfec_stream_probe(self.ctx, _ptr(src), n, _ptr(dst),
                                                      1 if copy else 0))

    # -- synthetic inputs ----------------------------------------------------
    def phase_backoff(self):
        """Large fixed batches left on the one-pass kernel (contention backoff)."""
        return self.lib.qfec_phase_backoff(self.ctx)

    def last_fixed_phased(self):
        """1 if the last device fixed-shape call ran the phased kernel, 0 the
        one-pass kernel, -1 none yet."""
        return self.lib.qfec_last_fixed_phased(self.ctx)

    def last_phase_grid(self):
        """Test hook: workgroups of the last phased launch (0: one-pass)."""
        return self.lib.qfec_debug_last_phase_grid(self.ctx)

    def debug_phase(self, extra, reset_backoff=True):
        """Test hook: extra workgroups in phased launches (forces the abandon
        path); reset_backoff clears the contention backoff."""
        return self._check(self.lib.qfec_debug_phase(self.ctx, extra, int(reset_backoff)))

    def debug_phase_min(self, min_phases):
        """Test hook: phased kernel from `min_phases` phases on (0 default,
        1 always, 0xFFFFFFFF never)."""
        return self._check(self.lib.qfec_debug_phase_min(self.ctx, min_phases))

    def async_ticket(self):
        """Ticket of the last ragged call if it was queued (QFEC_ASYNC), else 0."""
        return self.lib.qfec_async_ticket(self.ctx)

    def complete_ticket(self, ticket, wait=True):
        """Finish one queued op: 0 done, QFEC_PENDING (1) still running;
        raises its own error only."""
        rc = self.lib.qfec_complete_ticket(self.ctx, ticket, 1 if wait else 0)
        return rc if rc == 1 else self._check(rc)

    def service_warm(self):
        """qfec_service_warm: make sure the small-batch service's worker runs
        (an event loop's turn start); a no-op with the service off."""
        self._check(self.lib.qfec_service_warm(self.ctx))

    def debug_service(self, on=None, poison_next=False):
        """Small-batch service hook: on True / False enables / disables the
        resident worker (None leaves it); poison_next malforms the next job's
        ring entry (test of the ring-miss path); returns {launches, jobs, alive}."""
        st = (C.c_uint64 * 6)()
        mode = 2 if poison_next else (3 if on is None else int(bool(on)))
        self._check(self.lib.qfec_debug_service(self.ctx, mode, st))
        d = {"launches": st[0], "jobs": st[1], "alive": st[2]}
        if mode == 3:  # the registry's view: worker stream busy, us since last use
            d["stream_busy"], d["idle_us"], d["rotations"] = st[3], st[4], st[5]
        return d

    def debug_service_stamps(self, on=None):
        """Measurement hook: the worker's wall-clock stamps (10-ns ticks) of
        the last job: seen, entry, first group, all groups, fence, token."""
        st = (C.c_uint64 * 6)()
        self._check(self.lib.qfec_debug_service_stamps(self.ctx, -1 if on is None else int(bool(on)), st))
        return list(st)

    def debug_service_trace(self):
        """Measurement hook: the last service job end to end (44 words, see
        qfec.h qfec_debug_service_trace)."""
        st = (C.c_uint64 * 44)()
        self._check(self.lib.qfec_debug_service_trace(self.ctx, st))
        return list(st)

    def debug_service_feed(self, on):
        """Measurement hook: a native thread owning this context flushes
        one-group mapped batches back to back (on=True); on=False stops it and
        returns {jobs, wrong}."""
        st = (C.c_uint64 * 2)()
        self._check(self.lib.qfec_debug_service_feed(self.ctx, 1 if on else 0, st))
        return None if on else {"jobs": st[0], "wrong": st[1]}

    def debug_service_hold(self, hold):
        """Test hook: the service's followers wait at their start while held."""
        return self._check(self.lib.qfec_debug_service_hold(self.ctx, 1 if hold else 0))

    def debug_service_resident(self, ns):
        """Test hook: the worker's residency bound in ns (0: rotate at every
        job); returns the previous bound."""
        return int(self.lib.qfec_debug_service_resident(self.ctx, int(ns)))

    def debug_service_idle(self, us):
        """Test hook: the worker's idle time in us for later launches (default
        100); returns the previous value."""
        return int(self.lib.qfec_debug_service_idle(self.ctx, int(us)))

    def debug_phase_regsteps(self, on):
        """Test hook: phased launches with (True) or without their register-held steps."""
        return self._check(self.lib.qfec_debug_phase_regsteps(self.ctx, 1 if on else 0))

    def debug_other_service_cus(self):
        """Test hook: (CUs a phased launch here leaves to other contexts' workers, why-bits)."""
        why = C.c_uint32(0)
        n = self.lib.qfec_debug_other_service_cus(self.ctx, C.byref(why))
        return int(n), int(why.value)

    def debug_phase_reserve(self, cus):
        """Test hook: phased grids leave `cus` more CUs out (the CU-arbitration A/B)."""
        return self._check(self.lib.qfec_debug_phase_reserve(self.ctx, cus))

    def debug_phase_rtbatch(self, batch):
        """Test hook: the runtime-k phased body's load batch (16, 32; 0 = default 32)."""
        return self._check(self.lib.qfec_debug_phase_rtbatch(self.ctx, batch))

    def complete(self, wait=True):
        """Finish QFEC_ASYNC calls: 0 done, QFEC_PENDING (1) still running."""
        rc = self.lib.qfec_complete(self.ctx, 1 if wait else 0)
        return rc if rc == 1 else self._check(rc)

    def phase_abandons(self):
        """Phased fixed-shape launches that gave up their grid-wide meetings."""
        n = C.c_uint32(0)
        self._check(self.lib.qfec_phase_abandons(self.ctx, C.byref(n)))
        return n.value

    def synth_fixed(self, rows, k, L, g0, n_groups, seed, *, row_stride=None, group_stride=None):
        rs = L if row_stride is None else row_stride
        gs = k * rs if group_stride is None else group_stride
        return self._check(self.lib.qfec_synth_fixed(self.ctx, _ptr(rows), k, L, rs, gs, g0,
                                                     n_groups, seed))

    def synth_ragged(self, data, pkt_off, pkt_len, grp_ptr, g0, n_groups, seed):
        return self._check(self.lib.qfec_synth_ragged(self.ctx, _ptr(data), _ptr(pkt_off),
                                                      _ptr(pkt_len), _ptr(grp_ptr), g0,
                                                      n_groups, seed))


# -- v<=31 wire format (host-only C-ABI: no device, no context) -------------------
class FecHeader(C.Structure):
    """qfec_fec_header"""
    _fields_ = [("entropy_flag", C.c_uint8), ("fec_flag", C.c_uint8),
                ("in_fec_group", C.c_uint8), ("fec_group_offset", C.c_uint8)]


def _last_error():
    return load().qfec_last_error(None).decode()


def wire_write_private_header(entropy=False, fec=False, in_group=False, offset=0):
    """bytes written by qfec_wire_write_private_header (b"" on failure)."""
    h = FecHeader(int(entropy), int(fec), int(in_group), offset)
    buf = (C.c_uint8 * 4)()
    n = load().qfec_wire_write_private_header(C.byref(h), C.addressof(buf), 4)
    return bytes(buf[:n])


def wire_parse_private_header(data: bytes, version: int, packet_number: int):
    """(consumed, FecHeader) or (0, detailed_error)."""
    h = FecHeader()
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    n = load().qfec_wire_parse_private_header(C.addressof(buf), len(data), version,
                                              packet_number, C.byref(h))
    return (n, h) if n else (0, _last_error())


def wire_write_revived(revived, packet_number_length):
    arr = (C.c_uint64 * max(1, len(revived)))(*revived)
    cap = 1 + len(revived) * 8
    buf = (C.c_uint8 * cap)()
    n = load().qfec_wire_write_revived(C.addressof(arr), len(revived), packet_number_length,
                                       C.addressof(buf), cap)
    return bytes(buf[:n])


def wire_parse_revived(data: bytes, packet_number_length):
    """(consumed, [packet numbers]) or (0, detailed_error)."""
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    out = (C.c_uint64 * 256)()
    cnt = C.c_size_t(0)
    n = load().qfec_wire_parse_revived(C.addressof(buf), len(data), packet_number_length,
                                       C.addressof(out), C.byref(cnt))
    return (n, list(out[:cnt.value])) if n else (0, _last_error())


def wire_fec_packet_body(packet_number, fec_group, entropy, redundancy: bytes):
    red = (C.c_uint8 * max(1, len(redundancy))).from_buffer_copy(redundancy or b"\0")
    cap = 2 + len(redundancy)
    buf = (C.c_uint8 * cap)()
    n = load().qfec_wire_fec_packet_body(packet_number, fec_group, int(entropy),
                                         C.addressof(red), len(redundancy), C.addressof(buf), cap)
    return bytes(buf[:n])
