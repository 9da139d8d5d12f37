"""Static check of vector-memory / LDS wait counts in one kernel's gfx950
assembly (hipcc -S): inside each basic block, every VGPR that is the
destination of a load still outstanding (by the in-order vmcnt / LDS lgkmcnt
counters) must not be read or overwritten before an s_waitcnt retires it.
Blocks start from an empty state (cross-block hazards are not modelled).

Used on the ragged flat-window kernel pair whose sources are semantically
identical but one of which computes wrong parity ("code-
generation-dependent wrong results").
Usage: python tools/debug/waitcnt_check.py kernel.s"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(lines):
    issues = []
    vm, lgkm = [], []  # outstanding (line no, dest regs)
    for no, raw in enumerate(lines):
        line = raw.split(";")[0].strip()
        if not line or line.startswith("."):
            if re.match(r"^\.LBB|^\.L\w+:", line):
                vm, lgkm = [], []
            continue
        if line.endswith(":"):
            vm, lgkm = [], []
            continue
        op, _, rest = line.partition(" ")
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", rest)
            if m:
                n = int(m.group(1))
                vm = vm[len(vm) - n:] if n < len(vm) else vm
                if n == 0:
                    vm = []
            m = re.search(r"lgkmcnt\((\d+)\)", rest)
            if m:
                n = int(m.group(1))
                lgkm = lgkm[len(lgkm) - n:] if n < len(lgkm) else lgkm
                if n == 0:
                    lgkm = []
            continue
        if op.startswith("s_cbranch") or op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            vm, lgkm = [], []
            continue
        operands = [o.strip() for o in rest.split(",")] if rest else []
        is_load = op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load"))
        is_ds_ret = op.startswith("ds_") and ("read" in op or "bpermute" in op or "_rtn" in op
                                              or "swizzle" in op or "permute" in op)
        is_store = op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store")) \
            or (op.startswith("ds_") and not is_ds_ret)
        if is_store or op.startswith(("s_", "global_atomic", "buffer_atomic")):
            dst, srcs = set(), set().union(*[regs(o) for o in operands]) if operands else set()
        else:
            dst = regs(operands[0]) if operands else set()
            srcs = set().union(*[regs(o) for o in operands[1:]]) if len(operands) > 1 else set()
        for (lno, d) in vm + lgkm:
            if d & srcs:
                issues.append((no, f"reads v{sorted(d & srcs)} loaded at line {lno} (outstanding): {line}"))
            if d & dst and not (is_load or is_ds_ret):
                issues.append((no, f"overwrites v{sorted(d & dst)} loaded at line {lno}: {line}"))
        if is_load:
            vm.append((no, dst))
        elif is_ds_ret:
            lgkm.append((no, dst))
        elif op.startswith("ds_"):
            lgkm.append((no, set()))
        elif op.startswith(("global_store", "buffer_store", "global_atomic")):
            vm.append((no, set()))
    return issues


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().splitlines()
    iss = check(lines)
    for no, msg in iss[:50]:
        print(f"{no}: {msg}")
    print(f"{len(iss)} potential hazards")
