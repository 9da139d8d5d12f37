"""Generates tests/golden/wire_ref.npz: the REFERENCE QuicFramer's verdicts on
the v<=31 FEC wire cases of tests/wire_cases.py, so that the wire parity test
also runs where /root/reference (and so oracle/_ref/libref_framer.so) is
absent.  Run here:  python tests/golden/make_golden_wire.py

Every verdict comes from the reference's own framer compiled from its sources
(oracle/ref/Makefile -> oracle/_ref/libref_framer.so); nothing is restated."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import ref_framer as R  # noqa: E402
import wire_cases as W  # noqa: E402


def main():
    assert R.available(), "build oracle/_ref first (make -C oracle/ref)"
    rows = []
    for v, pn, body in W.private_header_cases():
        ph = R.public_header(v, pn, W.pn_len_for(pn))
        r = R.parse(v, R.encrypt(v, pn, ph + body, len(ph)))
        rows.append((v, pn, body, r["header_seen"], r["entropy_flag"], r["fec_flag"], r["error"],
                     r["detailed_error"]))
    n = len(rows)
    body = np.zeros((n, 8), np.uint8)
    blen = np.zeros(n, np.uint8)
    for i, row in enumerate(rows):
        body[i, :len(row[2])] = np.frombuffer(row[2], np.uint8)
        blen[i] = len(row[2])
    np.savez_compressed(
        os.path.join(ROOT, "tests", "golden", "wire_ref.npz"),
        version=np.array([r[0] for r in rows], np.int32),
        pn=np.array([r[1] for r in rows], np.uint64), body=body, body_len=blen,
        header_seen=np.array([r[3] for r in rows], np.int8),
        entropy=np.array([r[4] for r in rows], np.int8),
        fec=np.array([r[5] for r in rows], np.int8),
        error=np.array([r[6] for r in rows], np.int32),
        detail=np.array([r[7].encode() for r in rows], dtype="S80"))
    print(f"{n} private-header cases")


if __name__ == "__main__":
    main()
