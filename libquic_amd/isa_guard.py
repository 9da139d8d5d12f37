"""Build guard: find 64-bit VALU shifts that read their 32-bit shift amount
from the wave's last allocated VGPR, in gfx950 code.

tools/debug/last_vgpr_operand.hip measured on MI355X: `v_lshlrev_b64 vD,
vLAST, v[..]`, with vLAST the allocation's last VGPR (v55 of 56, v63 of 64),
shifts by the value of v0 instead in ~8% of executions when several waves
share a SIMD (0 with one wave per SIMD; 0 with the amount in v40; 0 for the
32-bit v_lshlrev_b32).  "Last" is the last register of the granule-rounded
allocation.  tools/debug/last_vgpr_ops.hip: v_lshlrev_b64 and v_lshrrev_b64
are affected (24% of executions at 8 waves/SIMD, the amount read as v0, never
v1); v_lshl_add_u64 (amount as src1), v_mad_u64_u32, v_cvt_f64_u32 and
v_mul_lo_u32 reading the last register are not.  v_ashrrev_i64 (same shifter,
not measured) is guarded too.  That is the round-1 ragged build's wrong result
(DESIGN.md §4).  build.build_lib() runs this over every libqfec.so it links
and refuses to install one that has such an instruction; the fix is to
change the kernel (a different register assignment, or no variable 64-bit
shift) — tests/test_isa_guard.py checks the installed library.

Input: assembly (.s, hipcc --save-temps) or a built library / code object
(.so / .co / .hsaco: its gfx950 code object is unbundled, disassembled with
llvm-objdump and its VGPR counts read from the AMDHSA metadata notes).

Usage: python -m libquic_amd.isa_guard file.{s,so,co} [...]
Exit status 1 if any kernel has one."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"

SHIFT64 = re.compile(r"^\s*(v_lshlrev_b64|v_lshrrev_b64|v_ashrrev_i64)\s+(v\[\d+:\d+\]),\s*(\S+),")


def _code_objects(path, tmp):
    """gfx950 code objects of a host library or executable — one per
    translation unit: its .hip_fatbin section is a concatenation of offload
    bundles — or [path] for a code object itself."""
    with open(path, "rb") as f:
        if f.read(4) != b"\x7fELF":
            raise ValueError(f"{path}: not ELF")
    hdr = subprocess.run([f"{LLVM}/llvm-readelf", "-h", path], capture_output=True, text=True)
    if "AMDGPU" in hdr.stdout or "EM_AMDGPU" in hdr.stdout:
        return [path]
    fb = os.path.join(tmp, "fb.bin")
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(tmp, "x")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, a in enumerate(starts):
        b = starts[i + 1] if i + 1 < len(starts) else len(data)
        part = os.path.join(tmp, f"bundle{i}.bin")
        with open(part, "wb") as f:
            f.write(data[a:b])
        co = os.path.join(tmp, f"gfx950_{i}.co")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={co}"], check=True, capture_output=True)
        out.append(co)
    return out


def _notes_and_dis(path, dis=True):
    notes, text = [], []
    with tempfile.TemporaryDirectory() as tmp:
        for co in _code_objects(path, tmp):
            notes.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                        capture_output=True, text=True).stdout)
            if dis:
                text.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True,
                                           capture_output=True, text=True).stdout)
    return notes, text


def private_segments(path):
    """{kernel: private (scratch) segment bytes} from a library / code object's
    AMDHSA metadata — a product kernel that spills to scratch is a
    performance bug (an array in bytes16_at once did: 4x slower)."""
    out = {}
    for notes in _notes_and_dis(path, dis=False)[0]:
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                out[name] = int(m.group(1))
    return out


def kernels_co(path):
    """yield (name, vgpr_count, [instruction lines]) from every code object of
    a library / executable / code object."""
    notes_all, dis_all = _notes_and_dis(path)
    for notes, dis in zip(notes_all, dis_all):
        vg, name = {}, None
        for line in notes.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s*\.vgpr_count:\s+(\d+)", line)
            if m and name:
                vg[name] = int(m.group(1))
        cur, body = None, []
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
            if m:
                if cur in vg:
                    yield cur, vg[cur], body
                cur, body = m.group(1), []
                continue
            if cur:
                body.append(line.split("//")[0].rstrip())
        if cur in vg:
            yield cur, vg[cur], body


def kernels(path):
    """yield (name, next_free_vgpr, [instruction lines])."""
    if not path.endswith(".s"):
        yield from kernels_co(path)
        return
    name, body, out = None, [], []
    for line in open(path):
        m = re.match(r"^(_Z\w+|\w+):\s*(;.*)?$", line)
        if m and not line.startswith(".L"):
            name, body = m.group(1), []
            continue
        if name and line.strip().startswith(".Lfunc_end"):
            out.append((name, body))
            name = None
            continue
        if name:
            body.append(line.split(";")[0].rstrip())
    vg = {}
    cur = None
    for line in open(path):
        m = re.match(r"\s*\.amdhsa_kernel\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s*\.amdhsa_next_free_vgpr\s+(\d+)", line)
        if m and cur:
            vg[cur] = int(m.group(1))
    for n, b in out:
        if n in vg:
            yield n, vg[n], b


GRANULE = 8  # gfx950 wave64 VGPR allocation granule


def scan(path):
    hits = []
    for name, nv, body in kernels(path):
        # the hardware allocates whole granules: the last register is the
        # granule-rounded count - 1 (a kernel using 69 VGPRs owns v0..v71)
        last = f"v{(nv + GRANULE - 1) // GRANULE * GRANULE - 1}"
        for i, l in enumerate(body):
            m = SHIFT64.match(l)
            if m and m.group(3) == last:
                hits.append((name, nv, l.strip()))
    return hits


def main(paths):
    bad = 0
    for p in paths:
        hits = scan(p)
        n_k = sum(1 for _ in kernels(p))
        print(f"{p}: {n_k} kernels, {len(hits)} 64-bit shifts with the amount in the last VGPR")
        for name, nv, l in hits:
            print(f"  {name} (VGPRs {nv}): {l}")
        bad += len(hits)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main(sys.argv[1:])
