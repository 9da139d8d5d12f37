"""ctypes binding of integration/connection_shim.cc (fec_conn_run): client /
server pairs of the patched reference QuicConnection at QUIC_VERSION_31 over
a lossy in-memory writer, FEC on the GPU.  Test / bench infrastructure: the
library is integration/_build/libquic_fec_patched.so (integration/build.py).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libquic_fec_patched.so")
# the same build over tests/cpp/cpu_qfec_stub.c (CPU parity in place of the
# GPU): lets the CPU suite run the connection path's FEC end to end
LIB_CPU = os.path.join(HERE, "_build", "libquic_fec_patched_cpustub.so")


class Params(C.Structure):
    _fields_ = [("version", C.c_int32), ("n_pairs", C.c_int32), ("group_size", C.c_int32),
                ("drop_every", C.c_int32), ("stream_len", C.c_uint64), ("batched", C.c_int32),
                ("max_turns", C.c_int32), ("fail_encode", C.c_int32),
                ("require_gpu", C.c_int32), ("no_end_flush", C.c_int32), ("reorder", C.c_int32),
                ("inject_unencrypted_fec", C.c_int32), ("close_mid_batch", C.c_int32),
                ("fec_option", C.c_int32)]


_U64 = ("data_packets_sent fec_packets_sent dropped revived groups_one_loss fec_groups_skipped "
        "retransmitted stream_bytes turns launches groups_encoded groups_revived").split()


class Result(C.Structure):
    _fields_ = ([(n, C.c_uint64) for n in _U64] +
                [("fec_wall_us", C.c_double), ("fec_host_us", C.c_double),
                 ("cpu_xor_us", C.c_double),
                 ("cpu_xor_groups", C.c_uint64), ("streams_ok", C.c_int32),
                 ("connected", C.c_int32), ("status", C.c_int32), ("detail", C.c_char * 256),
                 ("fec_wait_us", C.c_double), ("fec_launch_us", C.c_double),
                 ("debug_revived", C.c_uint64)] +
                [(n, C.c_uint64) for n in ("revived_reported acks_with_revived "
                                           "retransmitted_after_report retransmitted_of_revived "
                                           "protected_entropy_set").split()] +
                [(n, C.c_int32) for n in ("server_close_error client_close_error "
                                          "peer_saw_close closed_with_pending").split()] +
                [(n, C.c_double) for n in ("fec_tables_us fec_call_us "
                                           "fec_launch_us_max").split()] +
                [(n, C.c_uint64) for n in ("payloads_adopted payloads_copied "
                                           "slabs_allocated").split()])


_libs = {}


def lib(cpu_stub=False):
    path = LIB_CPU if cpu_stub else LIB
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build it with python integration/build.py")
        h = C.CDLL(path)
        h.fec_conn_run.restype = C.c_int
        h.fec_conn_run.argtypes = [C.POINTER(Params), C.POINTER(Result)]
        _libs[path] = h
    return _libs[path]


def run(n_pairs=1, group_size=10, drop_every=2, stream_len=100_000, batched=True,
        max_turns=20_000, fail_encode=False, require_gpu=False, version=31,
        end_flush=True, reorder=0, inject_unencrypted_fec=False, close_mid_batch=0, cpu_stub=False,
        fec_option=0) -> dict:
    """One simulated run; returns the result fields as a dict.  cpu_stub: the
    build whose qfec entry points are the CPU test stub (no GPU needed)."""
    p = Params(version=version, n_pairs=n_pairs, group_size=group_size, drop_every=drop_every,
               stream_len=stream_len, batched=int(batched), max_turns=max_turns,
               fail_encode=int(fail_encode), require_gpu=int(require_gpu),
               no_end_flush=int(not end_flush), reorder=reorder,
               inject_unencrypted_fec=int(inject_unencrypted_fec),
               close_mid_batch=close_mid_batch, fec_option=fec_option)
    r = Result()
    lib(cpu_stub).fec_conn_run(C.byref(p), C.byref(r))
    out = {n: getattr(r, n) for n, _ in Result._fields_}
    out["detail"] = r.detail.decode(errors="replace")
    return out
