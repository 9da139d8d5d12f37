"""Build the native library in-tree: libquic_amd/libqfec.so (gfx950).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container; the .so travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libqfec.so")
ARCH = os.environ.get("QFEC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["qfec_kernels.hip", "qpp_kernels.hip", "qent_kernels.hip", "qfec_capi.cpp", "quic_fec_group.cc",
           "quic_fec_wire.cc", "quic_fec_connection.cc"]
HEADERS = ["qfec_internal.h", "quic_fec_group.h", "quic_fec_wire.h", "quic_fec_connection.h"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libqfec.so)")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=cwd)


# Per-file code-generation flags.  The packet-protection kernels are LDS-
# lookup / VALU chains at 2 waves/SIMD (LDS-limited): the max-ILP machine
# scheduler issues a whole AES round's lookups before the first wait instead
# of groups of 8 with lgkmcnt(0) — measured +8% AES-GCM, +5-14% NULL,
# +3% ChaCha20-Poly1305 (profiles/round1/tune_gcm_g4.txt, tune_protect_g4.txt).
FILE_FLAGS = {"qpp_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}
# the host C++: a local that shadows a parameter is an error (round 4: the
# group offset shadowed the buffer offset in QuicFecSender::OnData)
for _h in ("qfec_capi.cpp", "quic_fec_group.cc", "quic_fec_wire.cc", "quic_fec_connection.cc"):
    FILE_FLAGS[_h] = ["-Wshadow", "-Werror=shadow"]


def build_lib(force: bool = False, extra_flags=()) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(ROOT, "include", "qfec.h"), __file__]
    if force or _stale(LIB, deps):
        objs = []
        for s in srcs:
            o = os.path.join(CSRC, "build", os.path.basename(s) + ".o")
            os.makedirs(os.path.dirname(o), exist_ok=True)
            if force or _stale(o, [s] + deps[len(srcs):]):
                _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                      "-I", os.path.join(ROOT, "include"),
                      *FILE_FLAGS.get(os.path.basename(s), []), *extra_flags, "-c", s, "-o", o])
            objs.append(o)
        tmp = LIB + ".tmp"
        # export the C-ABI (qfec_*) and the C++ host mirror (net::*) only
        vs = os.path.join(CSRC, "build", "exports.map")
        with open(vs, "w") as f:
            f.write('{\n  global:\n    qfec_*;\n    extern "C++" { net::*; };\n'
                    '  local: *;\n};\n')
        _run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", f"-Wl,--version-script={vs}",
              "-o", tmp, *objs])
        # gfx950: a 64-bit shift whose amount sits in the wave's last VGPR can
        # shift by v0 instead — never install such a build
        from libquic_amd import isa_guard
        hits = isa_guard.scan(tmp)
        if hits:
            os.remove(tmp)
            raise RuntimeError("libqfec.so: 64-bit shift amount in the last VGPR (gfx950 hazard, "
                               "DESIGN.md §4): " + "; ".join(f"{n} ({v} VGPRs): {l}"
                                                             for n, v, l in hits))
        os.replace(tmp, LIB)
    return LIB


CPP_TESTS = ["test_quic_fec_group", "test_quic_fec_connection", "bench_connection"]


def build_cpp_tests(force: bool = False) -> list:
    """tests/cpp/<name>: C++ host-mirror tests linked against libqfec.so."""
    outs = []
    bdir = os.path.join(ROOT, "tests", "cpp", "build")
    oracle_c = os.path.join(ROOT, "oracle", "qfec_oracle.c")
    oobj = os.path.join(bdir, "qfec_oracle.o")
    for name in CPP_TESTS:
        src = os.path.join(ROOT, "tests", "cpp", name + ".cc")
        out = os.path.join(bdir, name)
        if not os.path.exists(src):
            continue
        deps = [src, LIB, oracle_c] + [os.path.join(CSRC, h) for h in HEADERS]
        if force or _stale(out, deps):
            os.makedirs(bdir, exist_ok=True)
            if force or _stale(oobj, [oracle_c]):
                _run(["gcc", "-O2", "-std=c11", "-fPIC", "-c", oracle_c, "-o", oobj])
            _run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"),
                  "-I", CSRC, "-I", os.path.join(ROOT, "oracle"), src, oobj,
                  "-L", HERE, "-lqfec", "-Wl,-rpath,$ORIGIN/../../../libquic_amd",
                  "-Wl,-rpath-link,/opt/rocm/lib", "-lpthread", "-o", out])
        outs.append(out)
    return outs


# Measurement tools that compile against the library's headers or kernels
# (tools/tune): rebuilt whenever those change, so a tool never runs with a
# stale view of a class layout (round 4: host_cost built before a
# QuicFecGroup layout change corrupted its heap on the GPU box).
TOOLS = [("host_cost.cc", False), ("pcie_duplex.hip", True), ("phased_copy.hip", True),
         ("null_phased.hip", True)]


def build_tools(force: bool = False) -> list:
    outs = []
    tdir = os.path.join(ROOT, "tools", "tune")
    bdir = os.path.join(tdir, "build")
    for src_name, hip in TOOLS:
        src = os.path.join(tdir, src_name)
        out = os.path.join(bdir, os.path.splitext(src_name)[0])
        if not os.path.exists(src):
            continue
        deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + \
            [os.path.join(ROOT, "include", "qfec.h")]
        deps += [os.path.join(CSRC, "qfec_kernels.hip")] if hip else [LIB]
        if force or _stale(out, deps):
            os.makedirs(bdir, exist_ok=True)
            if hip:
                _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", src, "-o", out])
            else:
                _run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                      src, "-L", HERE, "-lqfec", "-Wl,-rpath,$ORIGIN/../../../libquic_amd",
                      "-Wl,-rpath-link,/opt/rocm/lib", "-o", out])
        outs.append(out)
    return outs


# the host C++ (payload arena, group bookkeeping, receive
# map, CSR builders, batcher) under AddressSanitizer + UBSan on the CPU,
# against tests/cpp/cpu_qfec_stub.c (test infrastructure: a CPU restatement of
# the C-ABI calls the host code makes; never part of libqfec.so).
# (ThreadSanitizer as well for the group test: worker threads fill groups
# whose arena slabs outlive them.)
SAN_TESTS = [("san", "test_quic_fec_group"), ("san", "test_quic_fec_connection"),
             ("tsan", "test_quic_fec_group"), ("san", "test_layout_guard")]
# per-test defines: the layout-guard test plays a caller built against a
# different quic_fec_group.h
SAN_DEFINES = {"test_layout_guard": ["-DQFEC_TEST_STALE_LAYOUT"]}
HOST_SRCS = ["quic_fec_group.cc", "quic_fec_wire.cc", "quic_fec_connection.cc"]
SAN_FLAGS = {
    "san": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
            "-fno-omit-frame-pointer", "-g", "-O1"],
    "tsan": ["-fsanitize=thread", "-g", "-O1"],
}


def build_cpp_sanitized(force: bool = False) -> list:
    outs = []
    bdir = os.path.join(ROOT, "tests", "cpp", "build")
    stub = os.path.join(ROOT, "tests", "cpp", "cpu_qfec_stub.c")
    oracle_c = os.path.join(ROOT, "oracle", "qfec_oracle.c")
    hosts = [os.path.join(CSRC, f) for f in HOST_SRCS]
    for kind, name in SAN_TESTS:
        flags = SAN_FLAGS[kind]
        src = os.path.join(ROOT, "tests", "cpp", name + ".cc")
        out = os.path.join(bdir, f"{kind}_{name}")
        deps = [src, stub, oracle_c] + hosts + [os.path.join(CSRC, h) for h in HEADERS]
        if force or _stale(out, deps):
            os.makedirs(bdir, exist_ok=True)
            objs = []
            for c in (stub, oracle_c):
                o = os.path.join(bdir, f"{kind}_{os.path.basename(c)}.o")
                _run(["gcc", "-std=c11", *flags, "-I", os.path.join(ROOT, "include"),
                      "-c", c, "-o", o])
                objs.append(o)
            # the test TU alone gets its defines; the host sources build as shipped
            tobj = os.path.join(bdir, f"{kind}_{name}.o")
            _run(["g++", "-std=c++17", "-Wall", *flags, *SAN_DEFINES.get(name, []),
                  "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-I", os.path.join(ROOT, "oracle"),
                  "-c", src, "-o", tobj])
            _run(["g++", "-std=c++17", "-Wall", *flags, "-I", os.path.join(ROOT, "include"),
                  "-I", CSRC, "-I", os.path.join(ROOT, "oracle"), tobj, *hosts, *objs,
                  "-lpthread", "-o", out])
        outs.append(out)
    return outs


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    build_cpp_tests(force="--force" in sys.argv)
    build_cpp_sanitized(force="--force" in sys.argv)
    build_tools(force="--force" in sys.argv)
