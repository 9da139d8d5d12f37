"""The drop-in check: integration/libquic_fec.patch
applied to the reference's own QUIC sources.

CPU: the patch applies to /root/reference's files and every patched
translation unit — quic_protocol, quic_framer, quic_packet_creator,
quic_connection — plus the FEC host code built against the reference's types
(-DQFEC_WITH_LIBQUIC) compiles (g++ -fsyntax-only), and the patched framer +
packet creator + FEC host code LINK with the rest of what they need from the
reference tree (-z defs): integration/build.py.

GPU: integration/_build/libquic_fec_patched.so — the patched reference
QuicPacketCreator sends a FEC-protected QUIC_VERSION_31 stream (FEC packets
from the GPU parity), one data packet in N is dropped, the patched reference
QuicFramer receives the rest and the revived packets (GPU revive, then
QuicFramer::ProcessRevivedPacket), and the stream must come out
byte-identical (integration/patched_shim.cc).
"""
import ctypes as C
import os

import pytest

from conftest import ROOT

INTEG = os.path.join(ROOT, "integration")
LIB = os.path.join(INTEG, "_build", "libquic_fec_patched.so")


def _builder():
    import importlib.util
    spec = importlib.util.spec_from_file_location("integration_build",
                                                  os.path.join(INTEG, "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_patch_names_only_the_hook_files():
    files = [l.split()[2][2:] for l in open(os.path.join(INTEG, "libquic_fec.patch"))
             if l.startswith("diff --git ")]
    core = "src/net/quic/core/"
    assert sorted(files) == sorted(core + f for f in (
        "quic_protocol.h", "quic_protocol.cc", "quic_framer.h", "quic_framer.cc",
        "quic_packet_creator.h", "quic_packet_creator.cc", "quic_packet_generator.h",
        "quic_connection.h", "quic_connection.cc", "quic_connection_stats.h",
        "quic_connection_stats.cc",
        # the v<=31 ack's revived-packets list: receive side records revivals,
        # send side stops retransmitting what the peer revived
        "quic_received_packet_manager.h", "quic_received_packet_manager.cc",
        "quic_sent_packet_manager.h", "quic_sent_packet_manager.cc"))


def test_patch_applies_and_every_unit_compiles():
    B = _builder()
    if not B.available():
        pytest.skip("no /root/reference here: the patch is checked where the reference is")
    B.prepare()
    res = B.syntax_check()
    assert {u for u, _, _ in res} >= {"quic_connection.cc", "quic_framer.cc",
                                      "quic_packet_creator.cc", "quic_fec_group.cc"}
    bad = [(u, e[-2000:]) for u, rc, e in res if rc != 0]
    assert not bad, bad


def test_patched_units_link():
    B = _builder()
    if not B.available():
        pytest.skip("no /root/reference here")
    B.prepare()
    assert os.path.exists(B.build_lib())  # -z defs: nothing left undefined


class E2E(C.Structure):
    _fields_ = [("data_packets_sent", C.c_uint64), ("fec_packets_sent", C.c_uint64),
                ("dropped", C.c_uint64), ("revived", C.c_uint64), ("stream_bytes", C.c_uint64),
                ("stream_ok", C.c_int32), ("framer_errors", C.c_int32),
                ("fec_header_ok", C.c_int32), ("status", C.c_int32), ("detail", C.c_char * 256)]


def _run(group_size, stream_len, drop_every):
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: build it with python integration/build.py")
    lib = C.CDLL(LIB)
    lib.fec_e2e_run.restype = C.c_int
    lib.fec_e2e_run.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, C.POINTER(E2E)]
    r = E2E()
    rc = lib.fec_e2e_run(31, group_size, stream_len, drop_every, C.byref(r))
    assert rc == 0, r.detail.decode()
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("group_size,stream_len,drop_every",
                         [(10, 400_000, 10), (2, 60_000, 2), (255, 800_000, 255),
                          (10, 100_000, 0), (7, 300_000, 13)])
def test_patched_libquic_end_to_end(group_size, stream_len, drop_every):
    r = _run(group_size, stream_len, drop_every)
    assert r.framer_errors == 0
    assert r.fec_header_ok == 1
    assert r.fec_packets_sent == -(-r.data_packets_sent // group_size), r.detail.decode()
    if drop_every:
        assert r.dropped > 0
    # a group revives iff it lost exactly one packet
    expect = 0
    if drop_every:
        lost = {i // group_size for i in range(r.data_packets_sent)
                if i % drop_every == drop_every // 2}
        per = {}
        for i in range(r.data_packets_sent):
            if i % drop_every == drop_every // 2:
                per[i // group_size] = per.get(i // group_size, 0) + 1
        expect = sum(1 for g in lost if per[g] == 1)
    assert r.revived == expect
    # every byte arrives iff every group lost at most one packet
    assert bool(r.stream_ok) == (r.revived == r.dropped)
