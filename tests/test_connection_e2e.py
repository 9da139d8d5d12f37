"""The patched reference QuicConnection end to end (SURVEY.md §8 a5 / f2;
VERDICT r2 "what's missing" 1-2): integration/connection_shim.cc runs client /
server pairs of the REFERENCE's QuicConnection (patched by
integration/libquic_fec.patch, linked from /root/reference with everything it
reaches, no stand-ins) at QUIC_VERSION_31 over a lossy in-memory writer.
Every client sends a stream through SendStreamData; the channel drops at
most one data packet per FEC group (never an FEC packet); the servers receive
through the real ProcessUdpPacket -> ProcessValidatedPacket ->
MaybeProcessRevivedPackets (quic_connection.cc:1286-1392) and must deliver
every stream byte-identical, with exactly the groups that lost one packet
revived on the GPU.

CPU (no device): the reference's own loss recovery alone (FEC off), and the
FEC path when no GPU work can run — every group goes without FEC
(fec_groups_skipped) and retransmission still delivers the stream.

The FEC cases run twice: on the GPU (`gpu`, libqfec.so) and in the CPU suite
(`cpustub`) over the same patched build linked against
tests/cpp/cpu_qfec_stub.c, a CPU restatement of the qfec entry points the host
code calls (test infrastructure) -- so the connection path's groups, payload
arena, zero-copy capture, revival and ack channel are checked on every CPU run
too (round 4: a send-side zero-copy bug reached the GPU box before any CPU
test could see it).
"""
import ctypes as C
import os

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "integration", "_build", "libquic_fec_patched.so")
LIB_CPU = os.path.join(ROOT, "integration", "_build", "libquic_fec_patched_cpustub.so")

# backend of the FEC cases: the GPU, or the CPU stub build
BACKENDS = [pytest.param(False, marks=pytest.mark.gpu, id="gpu"),
            pytest.param(True, id="cpustub")]


def _harness(cpu_stub=False):
    if not os.path.exists(LIB_CPU if cpu_stub else LIB):
        if os.path.isdir("/root/reference/src/net/quic/core"):
            pytest.fail(f"{LIB} missing: python integration/build.py")
        pytest.skip("the patched reference library is built where /root/reference is")
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "conn_harness", os.path.join(ROOT, "integration", "conn_harness.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _have_device():
    lib = C.CDLL(os.path.join(ROOT, "libquic_amd", "libqfec.so"))
    lib.qfec_create.restype = C.c_void_p
    lib.qfec_destroy.argtypes = [C.c_void_p]
    c = lib.qfec_create(0)
    if c:
        lib.qfec_destroy(c)
    return bool(c)


def _check_revived_channel(r):
    """The reference's entropy bits on FEC-protected packets and the v<=31
    ack's revived-packets list: protected packets carry the creator's random
    entropy bit (about half are 1), every ack still validates (no connection
    closed on "Invalid entropy": _check_common), every revived packet is
    reported to its sender in an ack, and no packet is retransmitted after an
    ack reported it revived (QuicSentPacketManager::MarkPacketNotRetransmittable)."""
    if r["data_packets_sent"] >= 64:
        frac = r["protected_entropy_set"] / r["data_packets_sent"]
        assert 0.3 < frac < 0.7, r
    assert r["retransmitted_after_report"] == 0, r
    if r["revived"]:
        assert r["acks_with_revived"] > 0, r
        assert 0 < r["revived_reported"] <= r["revived"], r


def _check_common(r, n):
    assert r["status"] == 0, r["detail"]
    assert r["connected"] == n, r["detail"]
    assert r["streams_ok"] == n, r


# ---- CPU ---------------------------------------------------------------------

@pytest.mark.parametrize("n,drop_every", [(1, 0), (1, 3), (8, 2)])
def test_reference_connection_loss_recovery_without_fec(n, drop_every):
    h = _harness()
    r = h.run(n_pairs=n, group_size=0, drop_every=drop_every, stream_len=150_000)
    _check_common(r, n)
    assert r["revived"] == 0 and r["fec_packets_sent"] == 0
    if drop_every:
        assert r["dropped"] > 0 and r["retransmitted"] >= r["dropped"]


def test_reference_connection_over_a_reordering_link():
    """The reordering link with FEC off: the reference's loss recovery alone
    (spurious retransmissions of late packets included) delivers every stream."""
    h = _harness()
    r = h.run(n_pairs=3, group_size=0, drop_every=3, stream_len=150_000, reorder=3)
    _check_common(r, 3)
    assert r["dropped"] > 0 and r["retransmitted"] >= r["dropped"]


@pytest.mark.parametrize("batched", [False, True])
def test_fec_without_device_skips_groups(batched):
    h = _harness()
    if _have_device():
        pytest.skip("a HIP device is present: the GPU tests cover this path (fail_encode)")
    r = h.run(n_pairs=2, group_size=10, drop_every=2, stream_len=120_000, batched=batched)
    _check_common(r, 2)
    assert r["fec_packets_sent"] == 0 and r["revived"] == 0
    assert r["fec_groups_skipped"] > 0
    assert r["dropped"] > 0 and r["retransmitted"] >= r["dropped"]
    # zero-copy capture: every protected packet was serialized (sender) and
    # decrypted (receiver) into an arena buffer its group adopted -- heap
    # arena without a device -- and no payload was copied
    assert r["payloads_copied"] == 0, r
    assert r["payloads_adopted"] >= r["data_packets_sent"] > 0, r


def test_unencrypted_fec_data_closes_the_connection():
    """An FEC packet that arrives at ENCRYPTION_NONE closes the connection with
    QUIC_UNENCRYPTED_FEC_DATA (quic_protocol.h:549-550; the rule OnStreamFrame
    applies to stream data), before its redundancy reaches any group; the
    sender never FEC-protects a packet at ENCRYPTION_NONE.  No GPU work is
    reached, so this runs on the CPU."""
    h = _harness()
    r = h.run(n_pairs=1, group_size=0, drop_every=0, stream_len=20_000,
              inject_unencrypted_fec=True)
    assert r["status"] == 0, r["detail"]
    assert r["server_close_error"] == 77, r  # QUIC_UNENCRYPTED_FEC_DATA
    assert r["connected"] == 0 and r["streams_ok"] == 0, r
    assert r["revived"] == 0, r


# ---- FEC on the GPU (gpu) and over the CPU stub (cpustub) --------------------

@pytest.mark.parametrize("stub", BACKENDS)
@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("group_size,drop_every,n", [(10, 2, 4), (2, 3, 2), (255, 1, 2),
                                                     (10, 0, 2)])
def test_connection_fec_revives_every_single_loss(batched, group_size, drop_every, n, stub):
    """Every group that lost one packet is revived unless the sender's own
    loss recovery got there first (the peer's STOP_WAITING then closes the
    group: CloseFecGroupsBefore); with 10-packet groups the FEC packet always
    wins in this simulation (deterministic: simulated clock, one turn per
    millisecond), with 255-packet groups the retransmission may."""
    h = _harness(stub)
    r = h.run(n_pairs=n, group_size=group_size, drop_every=drop_every, stream_len=300_000,
              batched=batched, require_gpu=True, cpu_stub=stub)
    _check_common(r, n)
    assert r["fec_groups_skipped"] == 0, r
    assert r["fec_packets_sent"] > 0
    if drop_every:
        assert r["dropped"] > 0
    # at most one loss per group, never the FEC packet
    assert r["dropped"] == r["groups_one_loss"], r
    assert r["revived"] <= r["dropped"] <= r["revived"] + r["retransmitted"], r
    # every revival reached the debug visitor (where a NetLog logger hooks in)
    assert r["debug_revived"] == r["revived"], r
    if group_size <= 10:
        assert r["revived"] == r["dropped"], r
    if batched:
        assert r["launches"] > 0
        assert r["groups_encoded"] == r["fec_packets_sent"], r
        assert r["groups_revived"] == r["revived"], r
    _check_revived_channel(r)
    # zero-copy capture on both sides: no protected payload copied
    assert r["payloads_copied"] == 0 and r["payloads_adopted"] >= r["data_packets_sent"], r
    print({k: r[k] for k in ("turns", "data_packets_sent", "fec_packets_sent", "dropped",
                             "revived", "retransmitted", "launches", "revived_reported",
                             "acks_with_revived", "retransmitted_of_revived",
                             "protected_entropy_set", "payloads_adopted", "payloads_copied")})


@pytest.mark.parametrize("stub", BACKENDS)
@pytest.mark.parametrize("option", [1, 2], ids=["FSTR", "FHDR"])
def test_session_fec_policy_by_connection_option(option, stub):
    """VERDICT r4 missing 4: the session's FEC policy (the historical
    QuicClientSessionBase::OnCryptoHandshakeEvent hook,
    quic_client_session_base.h:48) as a client connection option.  No
    EnableFecSending call: the client's QuicConfig sends kFSTR / kFHDR in its
    hello, the server's QuicConfig processes it, and the patched
    QuicConnection::SetFromConfig turns FEC sending on at both ends — the
    groups that lost one packet are revived as with the explicit call."""
    h = _harness(stub)
    r = h.run(n_pairs=2, group_size=0, drop_every=2, stream_len=200_000, batched=True,
              require_gpu=True, cpu_stub=stub, fec_option=option)
    _check_common(r, 2)
    assert r["fec_packets_sent"] > 0, r
    assert r["dropped"] > 0 and r["revived"] == r["dropped"], r
    # without the option (and without the call) FEC stays off
    r0 = h.run(n_pairs=2, group_size=0, drop_every=2, stream_len=200_000, batched=True,
               cpu_stub=stub, fec_option=0)
    _check_common(r0, 2)
    assert r0["fec_packets_sent"] == 0 and r0["revived"] == 0, r0


@pytest.mark.parametrize("stub", BACKENDS)
@pytest.mark.parametrize("reorder", [3, 7])
def test_connection_fec_over_a_reordering_link(reorder, stub):
    """Client->server packets reordered (adjacent pairs swapped, about one in
    `reorder` held back a turn, so FEC packets also arrive before the data
    they protect): streams still byte-identical, every drop repaired by a
    revival or a retransmission, every revival reported to the debug
    visitor.  A packet that is only LATE can be revived too — its group's FEC
    packet overtook it, as the historical receiver did — so revivals may
    exceed the drops here; the late original is then a duplicate."""
    h = _harness(stub)
    r = h.run(n_pairs=4, group_size=10, drop_every=2, stream_len=300_000, batched=True,
              require_gpu=True, reorder=reorder, cpu_stub=stub)
    _check_common(r, 4)
    assert r["fec_groups_skipped"] == 0 and r["fec_packets_sent"] > 0, r
    assert r["dropped"] > 0 and r["revived"] > 0, r
    assert r["dropped"] <= r["revived"] + r["retransmitted"], r
    assert r["debug_revived"] == r["revived"], r
    _check_revived_channel(r)
    print({k: r[k] for k in ("turns", "data_packets_sent", "fec_packets_sent", "dropped",
                             "revived", "retransmitted", "launches", "revived_reported",
                             "retransmitted_of_revived")})


@pytest.mark.parametrize("stub", BACKENDS)
def test_fec_alarm_closes_a_partial_group(stub):
    """A stream shorter than one group and no end-of-data close: only the FEC
    alarm (the group took no packet for max(1 ms, srtt/2)) can close the
    group and send its FEC packet.  The loss itself is repaired by whichever
    comes first, the revival or the sender's fast retransmit."""
    h = _harness(stub)
    r = h.run(n_pairs=1, group_size=200, drop_every=1, stream_len=20_000, batched=True,
              require_gpu=True, end_flush=False, cpu_stub=stub)
    _check_common(r, 1)
    assert r["fec_packets_sent"] == 1 and r["fec_groups_skipped"] == 0, r
    assert r["dropped"] == 1 and r["revived"] + r["retransmitted"] >= 1, r


@pytest.mark.parametrize("stub", BACKENDS)
def test_gpu_failure_goes_without_fec(stub):
    """Every FEC launch fails (qfec_debug_fail_launches): the groups go out
    without FEC packets (fec_groups_skipped), nothing is revived, and the
    reference's retransmission still delivers every stream — no connection
    is closed (it was OnUnrecoverableError in round 2)."""
    h = _harness(stub)
    r = h.run(n_pairs=3, group_size=10, drop_every=2, stream_len=150_000, batched=True,
              fail_encode=True, require_gpu=True, cpu_stub=stub)
    _check_common(r, 3)
    assert r["fec_packets_sent"] == 0 and r["revived"] == 0
    assert r["fec_groups_skipped"] > 0
    assert r["retransmitted"] >= r["dropped"] > 0


@pytest.mark.parametrize("stub", BACKENDS)
def test_batcher_batches_across_connections(stub):
    """64 connections on one batcher: each launch carries many connections'
    groups (one encode + one revive launch per loop turn)."""
    h = _harness(stub)
    n = 64
    r = h.run(n_pairs=n, group_size=10, drop_every=2, stream_len=60_000, batched=True,
              require_gpu=True, cpu_stub=stub)
    _check_common(r, n)
    assert r["dropped"] == r["revived"] > 0
    assert r["groups_encoded"] >= 4 * r["launches"], r
    _check_revived_channel(r)


@pytest.mark.gpu
def test_close_while_fec_packet_pending():
    """A batched connection closes while its group's FEC packet is still being
    computed: packets numbered after a pending FEC packet are held back, but
    the CONNECTION_CLOSE must leave at once (IsTerminationPacket) -- the peer
    learns of the close, and the pending group goes without FEC.  GPU only:
    the CPU stub completes every launch inside the call (nothing pends)."""
    h = _harness()
    r = h.run(n_pairs=2, group_size=10, drop_every=2, stream_len=150_000, batched=True,
              require_gpu=True, close_mid_batch=3)
    assert r["status"] == 0, r["detail"]
    assert r["closed_with_pending"] == 1, r
    assert r["peer_saw_close"] == 1, r
    assert r["client_close_error"] == 16, r  # QUIC_PEER_GOING_AWAY
    assert r["connected"] == 1 and r["streams_ok"] == 1, r  # the other pair is untouched
