"""The v<=31 ack's revived-packets list as the PATCHED reference framer
writes and reads it (integration/libquic_fec.patch: quic_framer.cc
AppendAckFrameAndTypeByte / ProcessAckFrame / GetAckFrameSize; VERDICT r3
"next" 1): the patched QuicConnection lists the packets it revived in its
acks, and the sender's QuicSentPacketManager stops retransmitting them.

Pinned by the UNPATCHED reference: what the patched framer writes is parsed
by the reference's own QuicFramer (oracle/_ref/libref_framer.so, compiled from
/root/reference unmodified), which reads the list's count and numbers
(quic_framer.cc:1477-1493) and must then find the PING frame written after
it; with no revived packet the packet is byte-identical to the reference
writer's own ack (its "FEC is not supported" zero count, :2311-2317).
CPU only.
"""
import ctypes as C
import os

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "integration", "_build", "libquic_fec_patched.so")
U64P = C.POINTER(C.c_uint64)


def _libs():
    from oracle import ref_framer as R
    if not os.path.exists(LIB) or not R.available():
        if os.path.isdir("/root/reference/src/net/quic/core"):
            pytest.fail("patched / reference framer libraries missing: python -c "
                        "'import __graft_entry__ as g; g.build()'")
        pytest.skip("built where /root/reference is")
    L = C.CDLL(LIB)
    L.fec_ack_build.restype = C.c_size_t
    L.fec_ack_build.argtypes = [C.c_int, C.c_uint64, C.c_uint64, U64P, U64P, C.c_size_t,
                                U64P, C.c_size_t, C.c_int, C.c_void_p, C.c_size_t]
    L.fec_ack_parse.restype = C.c_int
    L.fec_ack_parse.argtypes = [C.c_int, C.c_void_p, C.c_size_t, U64P, C.c_size_t,
                                C.POINTER(C.c_int), C.POINTER(C.c_uint64)]
    return L, R


def _arr(xs):
    return (C.c_uint64 * max(1, len(xs)))(*xs)


def build(L, version, pn, largest, missing, revived, ping=True, cap=1452):
    buf = (C.c_uint8 * cap)()
    n = L.fec_ack_build(version, pn, largest, _arr([m[0] for m in missing]),
                        _arr([m[1] for m in missing]), len(missing), _arr(revived), len(revived),
                        int(ping), C.addressof(buf), cap)
    assert n, "patched BuildDataPacket failed"
    return bytes(buf[:n])


def parse_patched(L, version, pkt):
    out = (C.c_uint64 * 512)()
    pings = C.c_int(0)
    largest = C.c_uint64(0)
    b = (C.c_uint8 * len(pkt)).from_buffer_copy(pkt)
    n = L.fec_ack_parse(version, C.addressof(b), len(pkt), out, 512, C.byref(pings),
                        C.byref(largest))
    assert n >= 0, "patched framer refused the packet"
    return sorted(out[:n]), pings.value, largest.value


CASES = [
    # (largest observed, missing [lo, hi) ranges, revived)
    (20, [(5, 6), (10, 12)], [5, 11]),
    (20, [(5, 6), (10, 12)], [5, 10, 11]),
    (300, [(7, 8)], [7]),                       # 2-byte largest observed
    (70_000, [(65_600, 65_610)], [65_601, 65_609]),  # 4-byte numbers
    (1 << 33, [((1 << 33) - 9, (1 << 33) - 3)], [(1 << 33) - 5]),  # 6-byte numbers
]


@pytest.mark.parametrize("largest,missing,revived", CASES)
def test_revived_list_read_by_the_reference(largest, missing, revived):
    L, R = _libs()
    pkt = build(L, 31, largest + 1, largest, missing, revived)
    r = R.parse(31, pkt)
    assert r["accepted"] == 1, r["detailed_error"]
    assert r["n_ack"] == 1 and r["n_ping"] == 1 and r["complete"] == 1, r
    assert r["ack_largest_observed"] == largest
    assert r["ack_missing_count"] == sum(hi - lo for lo, hi in missing)
    got, pings, lo = parse_patched(L, 31, pkt)
    assert got == sorted(revived) and pings == 1 and lo == largest


@pytest.mark.parametrize("largest,missing,revived", CASES)
def test_no_revived_is_the_reference_ack(largest, missing, revived):
    """Without revived packets the patched writer's ack is the reference's."""
    L, R = _libs()
    pn = largest + 1
    ours = build(L, 31, pn, largest, missing, [], ping=False)
    plain, ad = R.build(31, pn, 6, False, "ack", largest, missing)
    assert ours == R.encrypt(31, pn, plain, ad)
    assert parse_patched(L, 31, ours)[0] == []


def test_revived_list_capped_at_255_newest_first():
    """The count is one byte: of 300 revived packets the 255 newest are listed."""
    L, R = _libs()
    revived = list(range(1000, 1300))
    pkt = build(L, 31, 2001, 2000, [(1000, 1300)], revived)
    r = R.parse(31, pkt)
    assert r["accepted"] == 1 and r["n_ping"] == 1, r
    got, _, _ = parse_patched(L, 31, pkt)
    assert got == revived[-255:]


def test_revived_above_largest_observed_not_listed():
    L, R = _libs()
    pkt = build(L, 31, 31, 30, [(5, 6)], [5, 35])
    assert R.parse(31, pkt)["accepted"] == 1
    assert parse_patched(L, 31, pkt)[0] == [5]


def test_revived_list_truncated_to_the_packet():
    """A packet too small for every revived number lists as many as fit and
    the reference still parses it (the ack is the packet's only frame)."""
    L, R = _libs()
    revived = list(range(100_000, 100_200))          # 200 x 4-byte numbers
    pkt = build(L, 31, 200_001, 200_000, [(100_000, 100_200)], revived, ping=False,
                cap=400)
    assert len(pkt) <= 400
    r = R.parse(31, pkt)
    assert r["accepted"] == 1 and r["n_ack"] == 1, r
    got, _, _ = parse_patched(L, 31, pkt)
    assert 0 < len(got) < 200 and got == revived[-len(got):]


def test_v32_ack_has_no_revived_list():
    L, R = _libs()
    pkt = build(L, 32, 21, 20, [(5, 6)], [5])
    r = R.parse(32, pkt)
    assert r["accepted"] == 1 and r["n_ping"] == 1, r
    assert parse_patched(L, 32, pkt)[0] == []


def test_revived_list_property_vs_reference():
    """Random acks (missing sets over up to 1,000 packets, random revived
    subsets of them, 1- to 6-byte largest observed, packet capacities from
    200 B): the unpatched reference framer accepts every ack the patched
    writer produces, and the patched reader returns the NEWEST revived
    packets at or below the largest observed the ack carries -- all of them
    when they fit (at most 255)."""
    from hypothesis import given, settings, strategies as st, HealthCheck
    L, R = _libs()

    @settings(max_examples=150, deadline=None, suppress_health_check=list(HealthCheck))
    @given(st.integers(2, 2**40), st.lists(st.integers(1, 1000), min_size=1, max_size=300),
           st.data(), st.sampled_from([200, 400, 1452]), st.booleans())
    def check(largest, back, data, cap, ping):
        miss = sorted({largest - b for b in back if largest - b >= 1})
        if not miss:
            return
        # as [lo, hi) ranges
        ranges, lo = [], miss[0]
        for a, b in zip(miss, miss[1:] + [None]):
            if b != a + 1:
                ranges.append((lo, a + 1))
                lo = b
        revived = sorted(set(data.draw(st.lists(st.sampled_from(miss), max_size=300))))
        pkt = build(L, 31, largest + 1, largest, ranges, revived, ping=ping, cap=cap)
        r = R.parse(31, pkt)
        assert r["accepted"] == 1 and r["n_ack"] == 1, r
        if ping and r["n_ping"] == 0:
            # the ping did not fit after the ack (ack truncated to the packet)
            pass
        got, _, lo_written = parse_patched(L, 31, pkt)
        assert lo_written == r["ack_largest_observed"]
        want = sorted((x for x in revived if x <= lo_written), reverse=True)
        assert got == sorted(want[:len(got)])
        if len(pkt) + 8 < cap - 12:  # room was left: nothing was cut
            assert len(got) == min(255, len(want))

    check()
