"""Generate a bitsliced AES S-box circuit for the round-6 bitsliced AES-CTR
probe (tools/tune/tune_aes_bitslice.hip).

The S-box is computed as FIPS-197 defines it -- the multiplicative inverse in
GF(2^8) (x^8 + x^4 + x^3 + x + 1) followed by the affine map -- with the
inverse taken in the tower field GF(((2^2)^2)^2) (each level a polynomial
basis over the one below, y^2 + y + nu), where it is a short circuit of ANDs
and XORs.  The field isomorphism is found by searching the tower field for a
root of the AES polynomial; the basis changes in and out (the latter merged
with the affine map) are XOR networks.  Every gate is on 32-bit words (one bit
of 32 blocks each).  The circuit is then fused for gfx950's three-input
v_bitop3_b32 (a single-use inner gate folded into its user) and checked
against the S-box table for all 256 inputs before anything is written.

  python tools/tune/gen_bitslice_sbox.py > tools/tune/aes_bitslice_sbox.inc

No reference source is used: FIPS-197 section 5.1.1 defines the S-box; the
tower-field inverse is the textbook construction (a^-1 = conj(a) / N(a)).
"""
import itertools
import sys


# ---- GF(2^8), AES polynomial: the table the circuit must reproduce ----------
def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = (a << 1) ^ (0x11B if a & 0x80 else 0)
        b >>= 1
    return r


def ginv(a):
    if a == 0:
        return 0
    for b in range(1, 256):
        if gmul(a, b) == 1:
            return b
    raise AssertionError


def affine(b):
    r = 0x63
    for i in range(8):
        bit = ((b >> i) ^ (b >> ((i + 4) % 8)) ^ (b >> ((i + 5) % 8)) ^ (b >> ((i + 6) % 8)) ^
               (b >> ((i + 7) % 8))) & 1
        r ^= bit << i
    return r


SBOX = [affine(ginv(x)) for x in range(256)]
assert SBOX[0] == 0x63 and SBOX[1] == 0x7C and SBOX[0x53] == 0xED


# ---- tower field arithmetic on integers (to find the isomorphism) -----------
# GF(4): bits (a1 a0) = a1*w + a0, w^2 = w + 1
def m2(a, b):
    a1, a0, b1, b0 = a >> 1, a & 1, b >> 1, b & 1
    hh = a1 & b1
    return ((hh ^ (a1 & b0) ^ (a0 & b1)) << 1) | (hh ^ (a0 & b0))


NU4 = 2  # GF(16) = GF(4)[z]/(z^2 + z + w): w = 2 makes it irreducible
LAM = None  # GF(256) = GF(16)[y]/(y^2 + y + LAM), chosen below


def m4(a, b):
    a1, a0, b1, b0 = a >> 2, a & 3, b >> 2, b & 3
    hh = m2(a1, b1)
    return ((hh ^ m2(a1, b0) ^ m2(a0, b1)) << 2) | (m2(hh, NU4) ^ m2(a0, b0))


def m8(a, b):
    a1, a0, b1, b0 = a >> 4, a & 15, b >> 4, b & 15
    hh = m4(a1, b1)
    return ((hh ^ m4(a1, b0) ^ m4(a0, b1)) << 4) | (m4(hh, LAM) ^ m4(a0, b0))


def irreducible4(nu):
    return all(m2(z, z) ^ z ^ nu for z in range(4))


def irreducible8(lam):
    return all(m4(y, y) ^ y ^ lam for y in range(16))


assert irreducible4(NU4)
LAM = next(l for l in range(16) if irreducible8(l))


def tpow(a, n):
    r = 1
    for _ in range(n):
        r = m8(r, a)
    return r


# a root beta of x^8 + x^4 + x^3 + x + 1 in the tower field: x^i -> beta^i
BETA = next(b for b in range(2, 256)
            if tpow(b, 8) ^ tpow(b, 4) ^ tpow(b, 3) ^ b ^ 1 == 0)
COLS = [tpow(BETA, i) for i in range(8)]  # image of AES basis bit i


def to_tower(x):
    r = 0
    for i in range(8):
        if x >> i & 1:
            r ^= COLS[i]
    return r


INV_COLS = [next(x for x in range(256) if to_tower(x) == 1 << i) for i in range(8)]


def from_tower(t):
    r = 0
    for i in range(8):
        if t >> i & 1:
            r ^= INV_COLS[i]
    return r


for x in range(256):
    assert from_tower(to_tower(x)) == x
    for y in (3, 0x57, 0xCA):
        assert to_tower(gmul(x, y)) == m8(to_tower(x), to_tower(y))


# ---- circuit builder ----------------------------------------------------------
class C:
    def __init__(self):
        self.g = []  # (op, a, b): op in 'in', 'xor', 'and', 'not'

    def inp(self, i):
        self.g.append(("in", i, None))
        return len(self.g) - 1

    def _new(self, op, a, b):
        self.g.append((op, a, b))
        return len(self.g) - 1

    def xor(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        return self._new("xor", a, b)

    def and_(self, a, b):
        return self._new("and", a, b)

    def not_(self, a):
        return self._new("not", a, None)


c = C()
X = [c.inp(i) for i in range(8)]


def lin(bits_in, cols):
    """y = M x over GF(2): cols[i] = image of input bit i (8-bit int)."""
    out = []
    for j in range(8):
        acc = None
        for i in range(8):
            if cols[i] >> j & 1:
                acc = c.xor(acc, bits_in[i])
        out.append(acc)
    return out


# tower ops on lists of node ids (LSB first); None = constant 0
def x2(a, b):
    return [c.xor(a[0], b[0]), c.xor(a[1], b[1])]


def c_m2(a, b):
    a0, a1 = a
    b0, b1 = b
    hh = c.and_(a1, b1)
    ll = c.and_(a0, b0)
    mid = c.and_(c.xor(a0, a1), c.xor(b0, b1))  # = a1b1 + a0b0 + a1b0 + a0b1
    return [c.xor(hh, ll), c.xor(mid, ll)]  # lo = hh + ll, hi = a1b0+a0b1+hh = mid + ll


def c_sq2(a):  # (a1 w + a0)^2 = a1 w^2 + a0 = a1 w + (a1 + a0)
    return [c.xor(a[0], a[1]), a[1]]


def c_mulw(a):  # a * w: (a1 w + a0) w = a1 (w + 1) + a0 w = (a1 + a0) w + a1
    return [a[1], c.xor(a[0], a[1])]


def c_scale2(a, k):  # a * constant k in GF(4)
    if k == 1:
        return a
    if k == 2:
        return c_mulw(a)
    if k == 3:  # w^2 = w + 1
        return c_mulw(c_mulw(a))
    raise AssertionError


def c_m4(a, b):
    a0, a1, b0, b1 = a[:2], a[2:], b[:2], b[2:]
    hh = c_m2(a1, b1)
    ll = c_m2(a0, b0)
    mid = c_m2(x2(a0, a1), x2(b0, b1))
    lo = x2(c_scale2(hh, NU4), ll)
    hi = x2(mid, ll)
    return lo + hi


def c_sq4(a):  # (a1 z + a0)^2 = a1^2 z^2 + a0^2 = a1^2 (z + nu) + a0^2
    s1, s0 = c_sq2(a[2:]), c_sq2(a[:2])
    return x2(c_scale2(s1, NU4), s0) + s1


def c_scale4(a, k):  # a * constant k in GF(16), k = k1 z + k0
    k1, k0 = k >> 2, k & 3
    a0, a1 = a[:2], a[2:]
    # (a1 z + a0)(k1 z + k0) = a1k1 (z + nu) + (a1 k0 + a0 k1) z + a0 k0
    def sc(v, kk):
        return [None, None] if kk == 0 else c_scale2(v, kk)
    hh = sc(a1, k1)
    lo = x2(sc(hh, NU4) if k1 else [None, None], sc(a0, k0))
    hi = x2(x2(hh, sc(a1, k0)), sc(a0, k1))
    return lo + hi


def c_inv2(a):  # in GF(4) the inverse is the square
    return c_sq2(a)


def c_inv4(a):
    a0, a1 = a[:2], a[2:]
    # N = a1^2 nu + a1 a0 + a0^2 ; inv = (a1 N^-1) z + (a0 + a1) N^-1
    n = x2(x2(c_scale2(c_sq2(a1), NU4), c_m2(a1, a0)), c_sq2(a0))
    ni = c_inv2(n)
    return c_m2(x2(a0, a1), ni) + c_m2(a1, ni)


def c_inv8(a):
    a0, a1 = a[:4], a[4:]
    s1 = c_sq4(a1)
    n = [c.xor(p, q) for p, q in zip(c_scale4(s1, LAM), c_m4(a1, a0))]
    n = [c.xor(p, q) for p, q in zip(n, c_sq4(a0))]
    ni = c_inv4(n)
    lo = c_m4([c.xor(p, q) for p, q in zip(a0, a1)], ni)
    hi = c_m4(a1, ni)
    return lo + hi


T = lin(X, COLS)
I = c_inv8(T)
# out = affine(from_tower(I)) = A(M^-1 I) + 0x63: merged columns
AFF_COLS = []
for i in range(8):
    AFF_COLS.append(affine(INV_COLS[i]) ^ 0x63)
Y = lin(I, AFF_COLS)
Y = [c.not_(y) if (0x63 >> j) & 1 else y for j, y in enumerate(Y)]


# ---- simulate (all 256 inputs at once: bit x of input word i = bit i of x) --
def simulate(gates, outs):
    v = []
    for op, a, b in gates:
        if op == "in":
            w = 0
            for x in range(256):
                w |= ((x >> a) & 1) << x
            v.append(w)
        elif op == "xor":
            v.append(v[a] ^ v[b])
        elif op == "and":
            v.append(v[a] & v[b])
        elif op == "not":
            v.append(v[a] ^ ((1 << 256) - 1))
    return [v[o] for o in outs]


res = simulate(c.g, Y)
for x in range(256):
    got = sum(((res[j] >> x) & 1) << j for j in range(8))
    assert got == SBOX[x], (x, got, SBOX[x])


# ---- dead-gate removal, then bitop3 fusion -----------------------------------
def live_set(gates, outs):
    live = set()
    st = list(outs)
    while st:
        n = st.pop()
        if n in live:
            continue
        live.add(n)
        op, a, b = gates[n]
        if op != "in":
            st.append(a)
            if b is not None:
                st.append(b)
    return live


live = live_set(c.g, Y)
uses = {}
for n in live:
    op, a, b = c.g[n]
    if op != "in":
        for s in (a, b):
            if s is not None:
                uses[s] = uses.get(s, 0) + 1
for o in Y:
    uses[o] = uses.get(o, 0) + 100  # outputs stay materialised

# expression of each node over at most 3 leaves: fold a single-use non-input
# operand into its user while the leaf count stays <= 3
expr = {}  # node -> (leaves tuple, truth function over leaves)
OPS = {"xor": lambda p, q: p ^ q, "and": lambda p, q: p & q}


forced = set()  # single-use nodes materialised because their user could not fold them


def leaves_fn(n):
    op, a, b = c.g[n]
    if op == "in" or uses.get(n, 0) != 1 or n in forced:
        return (n,), (lambda *v: v[0])
    return expr[n]


order = sorted(live)
emit = []
for n in order:
    op, a, b = c.g[n]
    if op == "in":
        continue
    if op == "not":
        la, fa = leaves_fn(a)
        expr[n] = (la, (lambda fa: lambda *v: ~fa(*v) & 1)(fa))
        continue
    la, fa = leaves_fn(a)
    lb, fb = leaves_fn(b)
    lv = tuple(dict.fromkeys(la + lb))
    if len(lv) > 3:  # cannot fold: the operands become materialised values
        for s_ in (a, b):
            if c.g[s_][0] != "in":
                forced.add(s_)
        la, fa = (a,), (lambda *v: v[0])
        lb, fb = (b,), (lambda *v: v[0])
        lv = tuple(dict.fromkeys(la + lb))
    ia = [lv.index(x) for x in la]
    ib = [lv.index(x) for x in lb]
    f = (lambda fa, fb, ia, ib, g: lambda *v: g(fa(*[v[i] for i in ia]), fb(*[v[i] for i in ib])))(
        fa, fb, ia, ib, OPS[op])
    expr[n] = (lv, f)

# materialise: every node used more than once, every output
mat = [n for n in order if c.g[n][0] != "in" and (uses.get(n, 0) != 1 or n in forced)]
names = {X[i]: f"x[{i}]" for i in range(8)}
lines = []
for n in mat:
    lv, f = expr[n]
    ref = [names[x] if x in names else None for x in lv]
    assert None not in ref, "operand not materialised"
    if len(lv) == 1:
        tt = f(0) | (f(1) << 1)
        code = ref[0] if tt == 2 else f"~{ref[0]}"
    else:
        # v_bitop3_b32 truth table: bit (a<<2 | b<<1 | c) of the table, with
        # a = 0xF0, b = 0xCC, c = 0xAA
        srcs = ref + [ref[0]] * (3 - len(ref))
        tt = 0
        for a_ in (0, 1):
            for b_ in (0, 1):
                for c_ in (0, 1):
                    vals = (a_, b_, c_)[:len(lv)]
                    # unused positions must not matter: they repeat leaf 0
                    if len(lv) < 3 and any(vals[0] != v for v in (a_, b_, c_)[len(lv):]):
                        continue
                    bit = f(*vals) & 1
                    idx = (a_ << 2) | (b_ << 1) | c_
                    tt |= bit << idx
        # fill the don't-care rows consistently (leaf 0 repeated)
        full = 0
        for idx in range(8):
            a_, b_, c_ = idx >> 2 & 1, idx >> 1 & 1, idx & 1
            vals = (a_, b_, c_)
            if len(lv) == 2:
                vals = (a_, b_)
            elif len(lv) == 1:
                vals = (a_,)
            full |= (f(*vals) & 1) << idx
        code = f"QFEC_BOP3({srcs[0]}, {srcs[1]}, {srcs[2]}, 0x{full:02X})"
    names[n] = f"t{len(lines)}"
    lines.append(f"  const uint32_t t{len(lines)} = {code};")

# ---- re-simulate the fused program ------------------------------------------
env = {}
for i in range(8):
    w = 0
    for x in range(256):
        w |= ((x >> i) & 1) << x
    env[f"x[{i}]"] = w
M = (1 << 256) - 1


def bop3(a, b, cc, t):
    r = 0
    for idx in range(8):
        if t >> idx & 1:
            r |= (a if idx & 4 else ~a & M) & (b if idx & 2 else ~b & M) & (cc if idx & 1 else ~cc & M)
    return r


for ln in lines:
    lhs, rhs = ln.strip()[len("const uint32_t "):].rstrip(";").split(" = ")
    if rhs.startswith("QFEC_BOP3("):
        args = rhs[10:-1].split(", ")
        env[lhs] = bop3(env[args[0]], env[args[1]], env[args[2]], int(args[3], 16))
    elif rhs.startswith("~"):
        env[lhs] = ~env[rhs[1:]] & M
    else:
        env[lhs] = env[rhs]
for x in range(256):
    got = sum(((env[names[Y[j]]] >> x) & 1) << j for j in range(8))
    assert got == SBOX[x]

gates = sum(1 for n in live if c.g[n][0] != "in")
print("// Generated by tools/tune/gen_bitslice_sbox.py -- do not edit.")
print(f"// Bitsliced AES S-box (FIPS-197 5.1.1) through the tower field GF(((2^2)^2)^2):")
print(f"// {gates} two-input gates, fused into {len(lines)} v_bitop3_b32 / moves;")
print("// checked against the S-box table for all 256 inputs.")
print("// x[0..7]: the 8 input bit-words (bit 0 = LSB of the byte); y[0..7] out.")
print("// QFEC_BOP3(a, b, c, t): bit (a << 2 | b << 1 | c) of t (v_bitop3_b32).")
print("#define QFEC_SBOX_BITSLICED(x, y) \\")
print("  do { \\")
for ln in lines:
    print(ln + " \\")
for j in range(8):
    print(f"  (y)[{j}] = {names[Y[j]]}; \\")
print("  } while (0)")
sys.stderr.write(f"gates {gates}, fused ops {len(lines)}, beta {BETA:#x}, lambda {LAM}\n")
