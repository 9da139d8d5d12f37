"""Case generators for the v<=31 FEC wire rows (shared by
tests/test_wire_reference.py and tests/golden/make_golden_wire.py).

Every case is plain bytes: the parts the reference's QuicFramer sees (public
header + packet number from the reference's own AppendPacketHeader, then the
private header and body) are assembled by the caller."""
from __future__ import annotations

VERSIONS = (30, 31, 32, 33)  # the versions with a private flags byte (v <= 33)


def pn_len_for(pn: int) -> int:
    return 1 if pn < 256 else 2 if pn < 65536 else 4 if pn < (1 << 32) else 6


def private_header_cases():
    """(version, packet_number, private-header-and-body bytes): every flags
    byte value x offsets around the packet number x truncation."""
    for v in VERSIONS:
        for pn in (1, 2, 7, 255, 256, 1000):
            for flags in range(256):
                offs = sorted({0, 1, pn - 1, pn, pn + 1, 255} & set(range(256)))
                for off in offs:
                    yield v, pn, bytes([flags, off]) + bytes(6)
                yield v, pn, bytes([flags])  # offset byte missing when FEC_GROUP is set
    for v in VERSIONS:
        yield v, 5, b""  # no private flags byte at all


def revived_cases():
    """(largest_observed, missing intervals, revived list) for v31 ack frames
    (the revived list is only present when the ack has nacks)."""
    for lo in (200, 60000, 1 << 20, (1 << 33) + 5):
        for n in (0, 1, 2, 17, 200, 255):
            if 1 + n * pn_len_for(lo) > 1350:  # the packet must stay <= kMaxPacketSize
                continue
            rev = [1 + (lo - 3 - 7 * i) % (lo - 1) for i in range(n)]  # in [1, lo)
            yield lo, [(lo - 2, lo)], rev
