"""CPU tests of the drop-in boundary: libqfec.so loads, exports every symbol
include/qfec.h declares, the Python binding declares the same set, and the
no-GPU behaviour is a loud failure (no silent CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "qfec.h")
LIB = os.path.join(ROOT, "libquic_amd", "libqfec.so")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qfec_[a-z_0-9]+)\s*\(", src)))


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"


def test_exports_every_declared_symbol():
    syms = header_symbols()
    assert len(syms) >= 17
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (qfec_[a-z_0-9]+)$", out, flags=re.M))
    missing = [s for s in syms if s not in exported]
    assert not missing, f"declared but not exported: {missing}"
    lib = C.CDLL(LIB)
    for s in syms:
        assert getattr(lib, s) is not None


def test_binding_matches_header():
    from libquic_amd import qfec
    assert sorted(n for n, _, _ in qfec.SIGNATURES) == header_symbols()


def test_abi_constants():
    from libquic_amd import qfec
    lib = qfec.load()
    assert lib.qfec_abi_version() == 1
    assert lib.qfec_strerror(0) == b"QUIC_NO_ERROR"
    assert lib.qfec_strerror(-5) == b"QUIC_INVALID_FEC_DATA"  # quic_protocol.h:538
    assert lib.qfec_strerror(-1) == b"QUIC_INTERNAL_ERROR"
    hdr = open(HEADER).read()
    assert "#define QFEC_MAX_PACKET_SIZE 1452u" in hdr        # quic_protocol.h:66
    assert "#define QFEC_DEFAULT_MAX_PACKET_SIZE 1350u" in hdr  # quic_protocol.h:56
    assert "#define QFEC_MAX_GROUP_PACKETS 255u" in hdr


def _gpu_visible():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-device failure mode")
def test_no_device_fails_loudly():
    from libquic_amd import qfec
    lib = qfec.load()
    assert not lib.qfec_create(0)
    assert b"no HIP device" in lib.qfec_last_error(None)
    with pytest.raises(qfec.QfecError):
        qfec.Context(0)
    # null-context calls return QUIC_INTERNAL_ERROR, never crash
    assert lib.qfec_sync(None) == -1
    assert lib.qfec_encode_batch(None, None, 10, 1350, 1, None, 0) == -1
    # round 6: the calls that skip the device bind on their fast paths still
    # refuse a null context
    assert lib.qfec_complete_ticket(None, 1, 0) == -1
    assert lib.qfec_service_warm(None) == -1
    assert lib.qfec_encode_ragged(None, None, None, None, None, 1, None, None, None,
                                  qfec.QFEC_PTR_MAPPED | qfec.QFEC_ASYNC) == -1
    assert lib.qfec_debug_service_resident(None, 0) == 0


def test_oracle_not_linked_by_product():
    # the product library must not carry the oracle (no CPU fallback path)
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True, check=True).stdout
    assert "qo_" not in out
    for dirpath, _, files in os.walk(os.path.join(ROOT, "libquic_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".cc", ".h", ".hip")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.replace("oracle/", "").lower() or f == "build.py", f
