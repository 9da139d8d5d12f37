"""Control-flow-aware static check of vector-memory / LDS wait counts in one
kernel's gfx950 assembly (hipcc --save-temps): every path through the
kernel's basic blocks (branch targets and fall-throughs, loop back edges
included) is followed with the in-order vmcnt (loads and stores) and LDS
lgkmcnt counters, and every VGPR that is the destination of a load still
outstanding on SOME path must not be read or overwritten there before an
s_waitcnt retires it.  tools/debug/waitcnt_check.py did the same inside one
basic block only.

Pending loads are merged over all paths into a block (a fixed point over
loop back edges); a path the program can never take (e.g. a branch
whose condition is fixed by an earlier one) can still be reported, so every
finding is checked by hand against the listing.

Usage: python tools/debug/waitcnt_cfg.py kernel.s SYMBOL"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
LOADS = ("global_load", "buffer_load", "flat_load", "scratch_load")
STORES = ("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic",
          "buffer_atomic", "flat_atomic")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def function(path, sym):
    """[(line_no, text)] of the function body, labels kept."""
    out, on = [], False
    for no, raw in enumerate(open(path), 1):
        line = raw.split(";")[0].strip()
        if raw.startswith(sym + ":"):
            on = True
            continue
        if not on:
            continue
        if line.startswith(".Lfunc_end"):
            break
        if not line or (line.startswith(".") and not line.endswith(":")):
            continue
        out.append((no, line))
    return out


def blocks(body):
    """label -> (first index, last index); successor lists."""
    starts = [0]
    for i, (_, l) in enumerate(body):
        if l.endswith(":"):
            starts.append(i)
        op = l.split(" ")[0]
        if op.startswith("s_cbranch") or op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            starts.append(i + 1)
    starts = sorted(set(s for s in starts if s < len(body)))
    label_at = {l[:-1]: i for i, (_, l) in enumerate(body) if l.endswith(":")}
    bl = []
    for j, s in enumerate(starts):
        e = starts[j + 1] if j + 1 < len(starts) else len(body)
        bl.append((s, e))
    start_to_block = {s: j for j, (s, _) in enumerate(bl)}
    succ = []
    for j, (s, e) in enumerate(bl):
        last = body[e - 1][1]
        op, _, rest = last.partition(" ")
        out = []
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = rest.strip()
            out.append(start_to_block[label_at[tgt]])
        if op != "s_branch" and op not in ("s_endpgm", "s_setpc_b64") and j + 1 < len(bl):
            out.append(j + 1)
        succ.append(out)
    return bl, succ


# State per counter: VGPR -> (ops issued after the load that writes it, load
# lines).  s_waitcnt xcnt(N) leaves at most N ops outstanding, and the counters
# retire in order, so a register with >= N younger ops is complete.  At a join
# the smaller count wins (fewer younger ops: harder to retire) — a finite
# lattice, so the worklist reaches a fixed point.
CAP = 64


def retire(st, n):
    return {r: v for r, v in st.items() if v[0] < n}


def issue(st, dst, no):
    out = {r: (min(c + 1, CAP), ls) for r, (c, ls) in st.items()}
    for r in dst:
        out[r] = (0, frozenset([no]))
    return out


def join(a, b):
    out = dict(a)
    for r, (c, ls) in b.items():
        if r in out:
            c0, l0 = out[r]
            out[r] = (min(c0, c), l0 | ls)
        else:
            out[r] = (c, ls)
    return out


def step(line, state, issues, no):
    vm, lgkm = state
    op, _, rest = line.partition(" ")
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", rest)
        if m:
            vm = retire(vm, int(m.group(1)))
        m = re.search(r"lgkmcnt\((\d+)\)", rest)
        if m:
            lgkm = retire(lgkm, int(m.group(1)))
        return vm, lgkm
    if line.endswith(":") or op.startswith("s_"):
        return vm, lgkm
    operands = [o.strip() for o in rest.split(",")] if rest else []
    is_load = op.startswith(LOADS)
    is_ds_ret = op.startswith("ds_") and ("read" in op or "bpermute" in op or "_rtn" in op
                                          or "swizzle" in op or "permute" in op)
    is_store = op.startswith(STORES) or (op.startswith("ds_") and not is_ds_ret)
    if is_store:
        dst, srcs = set(), set().union(*[regs(o) for o in operands]) if operands else set()
    else:
        dst = regs(operands[0]) if operands else set()
        srcs = set().union(*[regs(o) for o in operands[1:]]) if len(operands) > 1 else set()
    for pend in (vm, lgkm):
        for r in srcs & pend.keys():
            issues.add((no, f"reads v{r} of the load at line(s) {sorted(pend[r][1])}, "
                            f"outstanding on some path: {line}"))
        if not (is_load or is_ds_ret):
            for r in dst & pend.keys():
                issues.add((no, f"overwrites v{r} of the load at line(s) {sorted(pend[r][1])}, "
                                f"outstanding on some path: {line}"))
    if is_load or op.startswith(STORES):
        vm = issue(vm, dst if is_load else set(), no)
        # a new load's destination is no longer pending from older loads
    elif op.startswith("ds_"):
        lgkm = issue(lgkm, dst if is_ds_ret else set(), no)
    return vm, lgkm


def check(path, sym):
    body = function(path, sym)
    bl, succ = blocks(body)
    issues = set()
    entry = [None] * len(bl)
    entry[0] = ({}, {})
    work = [0]
    while work:
        b = work.pop()
        st = entry[b]
        s, e = bl[b]
        for i in range(s, e):
            no, line = body[i]
            st = step(line, st, issues, no)
        for nb in succ[b]:
            if entry[nb] is None:
                new = st
            else:
                new = (join(entry[nb][0], st[0]), join(entry[nb][1], st[1]))
                if new == entry[nb]:
                    continue
            entry[nb] = new
            work.append(nb)
    return sorted(issues), len(bl)


if __name__ == "__main__":
    iss, n_blocks = check(sys.argv[1], sys.argv[2])
    for no, msg in iss[:60]:
        print(f"{no}: {msg}")
    print(f"{len(iss)} potential hazards ({n_blocks} blocks)")
