"""v<=31 FEC wire rows against the
REFERENCE's own QuicFramer.

The product side is the host C-ABI qfec_wire_* (include/qfec.h) over
libquic_amd/csrc/quic_fec_wire.cc.  The reference side is
oracle/_ref/libref_framer.so: quic_framer.cc and what it links, compiled from
/root/reference unmodified (oracle/ref/Makefile, release build; test
infrastructure).  Packets are assembled from the reference's own public header
(AppendPacketHeader), NULL-encrypted by the reference (EncryptInPlace) and
parsed by the reference (ProcessPacket -> ProcessAuthenticatedHeader
quic_framer.cc:1102-1141 / ProcessAckFrame :1477-1493).

Where the reference library is absent (a checkout without /root/reference),
the committed verdicts in tests/golden/wire_ref.npz (made by the reference:
tests/golden/make_golden_wire.py) pin the private-header parser instead.
CPU only: the wire code touches no device.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_npz
import wire_cases as W

QUIC_INVALID_PACKET_HEADER = 3   # quic_protocol.h:532
QUIC_INVALID_ACK_DATA = 9        # quic_protocol.h:566
PING_FRAME = 7                   # quic_protocol.h:266


def _ref():
    from oracle import ref_framer as R
    if not R.available():
        pytest.skip("oracle/_ref/libref_framer.so not built (no /root/reference here); "
                    "test_private_header_vs_reference_fixture covers the parser")
    return R


def _q():
    from libquic_amd import qfec
    return qfec


def _check_private_header(q, v, pn, body, seen, ent, fec, err, detail):
    n, h = q.wire_parse_private_header(body, v, pn)
    if seen:
        assert n in (1, 2), (v, pn, body.hex(), h)
        assert (h.entropy_flag, h.fec_flag) == (ent, fec), (v, pn, body.hex())
        # consumed: the offset byte exactly when the FEC_GROUP bit is set
        assert n == (2 if body[0] & 0x02 else 1)
        if n == 2:
            assert h.in_fec_group == 1 and h.fec_group_offset == body[1] < pn
    else:
        assert n == 0, (v, pn, body.hex())
        assert err == QUIC_INVALID_PACKET_HEADER
        assert h == detail, (v, pn, body.hex(), h, detail)


def test_private_header_vs_reference_framer():
    """Every private-flags byte x offsets around the packet number x truncation,
    v30-v33: accept/reject, entropy/FEC flags and the detailed error string of
    our parser equal the reference framer's, case by case."""
    R, q = _ref(), _q()
    n = 0
    for v, pn, body in W.private_header_cases():
        ph = R.public_header(v, pn, W.pn_len_for(pn))
        r = R.parse(v, R.encrypt(v, pn, ph + body, len(ph)))
        _check_private_header(q, v, pn, body, r["header_seen"], r["entropy_flag"],
                              r["fec_flag"], r["error"], r["detailed_error"])
        n += 1
    assert n > 30000


def test_private_header_vs_reference_fixture():
    """The same comparison against the reference's committed verdicts."""
    q = _q()
    g = load_npz("wire_ref.npz")
    assert len(g["version"]) > 30000
    for i in range(len(g["version"])):
        body = bytes(g["body"][i, :g["body_len"][i]])
        _check_private_header(q, int(g["version"][i]), int(g["pn"][i]), body,
                              int(g["header_seen"][i]), int(g["entropy"][i]), int(g["fec"][i]),
                              int(g["error"][i]), g["detail"][i].decode())


def test_fixture_matches_live_reference():
    """The fixture is what the reference says now (regenerate on a mismatch)."""
    R = _ref()
    g = load_npz("wire_ref.npz")
    for i in range(0, len(g["version"]), 97):
        v, pn = int(g["version"][i]), int(g["pn"][i])
        body = bytes(g["body"][i, :g["body_len"][i]])
        ph = R.public_header(v, pn, W.pn_len_for(pn))
        r = R.parse(v, R.encrypt(v, pn, ph + body, len(ph)))
        assert (r["header_seen"], r["entropy_flag"], r["fec_flag"], r["error"],
                r["detailed_error"]) == (g["header_seen"][i], g["entropy"][i], g["fec"][i],
                                         g["error"][i], g["detail"][i].decode())


def test_private_header_writer_vs_reference():
    """Our writer (a3's header half): the reference parses every header we
    write back to the same fields; and for a packet outside any group our byte
    equals the one the reference's own AppendPacketHeader writes."""
    R, q = _ref(), _q()
    for v in (30, 31):
        for pn in (3, 300):
            for ent in (0, 1):
                for fec in (0, 1):
                    for grp in (0, 1):
                        for off in (0, 1, 2, pn - 1 if pn < 256 else 255):
                            hb = q.wire_write_private_header(ent, fec, grp, off)
                            if fec and not grp:
                                assert hb == b""  # an FEC packet always names its group
                                continue
                            assert len(hb) == 1 + grp
                            ph = R.public_header(v, pn, W.pn_len_for(pn))
                            r = R.parse(v, R.encrypt(v, pn, ph + hb + bytes(4), len(ph)))
                            assert r["header_seen"] == 1 and r["error"] == 0
                            assert (r["entropy_flag"], r["fec_flag"]) == (ent, fec)
            for ent in (False, True):
                plain, ad = R.build(v, pn, W.pn_len_for(pn), ent, "ping")
                assert plain[ad:ad + 1] == q.wire_write_private_header(ent, False, False, 0)


@pytest.mark.parametrize("red_len", [1, 16, 1350, 1452])
def test_fec_packet_body_vs_reference(red_len):
    """SerializeFecPacketBody (a3): the reference framer takes the packet as an
    FEC packet of the right group; out-of-range groups are refused by both."""
    R, q = _ref(), _q()
    rng = np.random.default_rng(red_len)
    red = rng.integers(0, 256, red_len, dtype=np.uint8).tobytes()
    for pn, grp in ((11, 1), (256, 1), (1000, 745), (70000, 69999)):
        for ent in (False, True):
            body = q.wire_fec_packet_body(pn, grp, ent, red)
            assert len(body) == 2 + red_len and body[2:] == red
            ph = R.public_header(31, pn, W.pn_len_for(pn))
            r = R.parse(31, R.encrypt(31, pn, ph + body, len(ph)))
            assert r["accepted"] == 1 and r["header_seen"] == 1 and r["error"] == 0
            assert r["fec_flag"] == 1 and r["entropy_flag"] == int(ent)
            n, h = q.wire_parse_private_header(body, 31, pn)
            assert n == 2 and pn - h.fec_group_offset == grp
    for pn, grp in ((10, 0), (10, 11), (300, 44)):  # offset >= pn or > 255
        assert q.wire_fec_packet_body(pn, grp, False, red) == b""
    assert q.wire_fec_packet_body(11, 1, False, bytes(1453)) == b""  # > kMaxPacketSize
    # v32+: the reference refuses the FEC bits themselves
    ph = R.public_header(32, 11, 1)
    r = R.parse(32, R.encrypt(32, 11, ph + q.wire_fec_packet_body(11, 1, False, red), len(ph)))
    assert r["header_seen"] == 0 and r["detailed_error"] == "Illegal private flags value."


def test_revived_list_writer_vs_reference():
    """a6 write side: the reference's v31 ack = its v32 ack + the revived list,
    and that tail is byte-equal to our WriteRevivedPackets([])
    (quic_framer.cc:2307-2317 writes an empty list)."""
    R, q = _ref(), _q()
    for lo, miss, _ in W.revived_cases():
        p31, ad31 = R.build(31, 9, 1, True, "ack", lo, miss)
        p32, ad32 = R.build(32, 9, 1, True, "ack", lo, miss)
        assert ad31 == ad32 and p31[:len(p32)] == p32
        assert p31[len(p32):] == q.wire_write_revived([], W.pn_len_for(lo))


def test_revived_list_parser_vs_reference():
    """a6 read side: a v31 ack carrying OUR revived list, then a PING frame.
    The reference accepts it and sees the PING exactly when the list's length
    is right; our parser consumes the same bytes and returns the numbers.
    Truncated lists: both refuse with the same detailed error."""
    R, q = _ref(), _q()
    for lo, miss, rev in W.revived_cases():
        pnl = W.pn_len_for(lo)
        plain, ad = R.build(31, 9, 1, False, "ack", lo, miss)
        assert plain[-1] == 0  # the reference's empty revived list
        lst = q.wire_write_revived(rev, pnl)
        assert len(lst) == 1 + len(rev) * pnl
        pkt = plain[:-1] + lst + bytes([PING_FRAME])
        r = R.parse(31, R.encrypt(31, 9, pkt, ad))
        assert r["accepted"] == 1 and r["n_ack"] == 1 and r["n_ping"] == 1, (lo, len(rev), r)
        assert r["ack_largest_observed"] == lo
        n, got = q.wire_parse_revived(lst + bytes([PING_FRAME]), pnl)
        assert n == len(lst) and got == rev
        # truncations: every cut inside the list
        for cut in sorted({1, len(lst) - 1, len(lst) // 2} - {0, len(lst)}):
            if cut <= 0 or cut >= len(lst):
                continue
            bad = plain[:-1] + lst[:cut]
            r = R.parse(31, R.encrypt(31, 9, bad, ad))
            assert r["accepted"] == 0 and r["error"] == QUIC_INVALID_ACK_DATA
            n, err = q.wire_parse_revived(lst[:cut], pnl)
            assert n == 0 and err == r["detailed_error"] == "Unable to read revived packet."
        # the count byte itself missing
        r = R.parse(31, R.encrypt(31, 9, plain[:-1], ad))
        assert r["accepted"] == 0 and r["error"] == QUIC_INVALID_ACK_DATA
        n, err = q.wire_parse_revived(b"", pnl)
        assert n == 0 and err == r["detailed_error"] == "Unable to read num revived packets."
