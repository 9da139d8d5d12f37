"""Offline analysis of tools/debug/anomaly_diag.hip's per-window dump (the
`W g .. t ..` lines: got / want / parity / every received packet's window)
for the failing round-1 ragged build.

Tests, per wrong 16-B accumulator window:
  1. is the difference a GF(2) combination of the packets' windows (a window
     XOR lost or applied twice)?
  2. is it `(w1 << k) & ~w0` for one packet's window (w0 / w1 its low / high
     8 bytes): the kernel's funnel shift `r0 = (w0 >> s) | ((w1 << 1) << v55)`
     with v55 = 63 (a full window) replaced by some other amount k - 1?
  3. if so, where did k - 1 come from: the low 6 bits of which loaded dword?
Usage: python tools/debug/anomaly_analyze.py gpurun_out/anom/diag.txt"""
import collections
import itertools
import re
import sys

M = (1 << 64) - 1


def x(a, b):
    return bytes(p ^ q for p, q in zip(a, b))


def load(path):
    rows = collections.defaultdict(list)
    for l in open(path):
        if not l.startswith("W "):
            continue
        m = re.match(r"W g (\d+) t (\d+) got (\w+) want (\w+) par (\w+)(.*)", l)
        g, t = int(m.group(1)), int(m.group(2))
        got, want, par = [bytes.fromhex(m.group(i)) for i in (3, 4, 5)]
        cs = [(int(r), int(f), bytes.fromhex(h))
              for r, f, h in re.findall(r"c(\d+):(\d+):(\w+)", m.group(6))]
        rows[g].append((t, got, want, par, cs))
    return rows


def main(path):
    rows = load(path)
    n_win = n_hi = n_gf2 = n_shift = 0
    slots = collections.Counter()
    src = collections.Counter()
    for g, ws in rows.items():
        for t, got, want, par, cs in ws:
            d = x(got, want)
            if not any(d):
                continue
            n_win += 1
            n_hi += any(d[8:])
            for k in range(1, len(cs) + 1):
                hit = False
                for sub in itertools.combinations(range(len(cs)), k):
                    acc = bytes(16)
                    for i in sub:
                        acc = x(acc, cs[i][2])
                    if acc == d:
                        hit = True
                        break
                if hit:
                    n_gf2 += 1
                    break
            dl = int.from_bytes(d[:8], "little")
            for r, f, c in cs:
                lo = int.from_bytes(c[:8], "little")
                hi = int.from_bytes(c[8:], "little")
                k = next((kk for kk in range(1, 64)
                          if ((hi << kk) & M) & ~lo == dl or ((hi << kk) & M) == dl), None)
                if k is None:
                    continue
                n_shift += 1
                slots[(f // 64) % 4] += 1
                dw = [int.from_bytes(c[4 * j:4 * j + 4], "little") & 63 for j in range(4)]
                src[tuple(j for j in range(4) if dw[j] == k - 1)] += 1
                break
    print(f"{len(rows)} dumped groups, {n_win} wrong windows, {n_hi} with a wrong high half")
    print(f"GF(2) combination of packet windows (lost / doubled XOR): {n_gf2}")
    print(f"(w1 << k) & ~w0 of one packet's window (wrong funnel-shift amount): {n_shift}")
    print(f"  by unroll slot of that window's wave-iteration: {dict(sorted(slots.items()))}")
    print("  k - 1 equals the low 6 bits of loaded dword(s) "
          f"{dict(sorted(src.items(), key=lambda kv: -kv[1]))}")


if __name__ == "__main__":
    main(sys.argv[1])
