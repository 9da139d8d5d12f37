"""Apply integration/libquic_fec.patch to the reference's QUIC sources and
build them together with the MI355X FEC host code — the drop-in check
(INTEGRATION.md).

  1. copy the patched files' originals from /root/reference/src into
     integration/_build/src (never into the repository: _build/ is
     git-ignored) and apply the patch with `patch -p1`, as the reference's own
     patch/ convention does;
  2. drop libquic_amd/csrc/quic_fec_{group,wire,connection}.{h,cc} into
     src/net/quic/core/ next to them, as a maintainer would;
  3. `g++ -fsyntax-only` every patched translation unit and the FEC host code
     (-DQFEC_WITH_LIBQUIC: the reference's own QuicPacketHeader, StringPiece,
     EncryptionLevel) against the reference headers;
  4. link the patched framer + packet creator + QuicConnection + the FEC host
     code + what they reach in the reference tree (packet generator, packet
     managers, congestion control, config, base/metrics: -z defs, no
     stand-ins) into integration/_build/libquic_fec_patched.so (C API:
     integration/patched_shim.cc — creator + framer — and
     integration/connection_shim.cc — QuicConnection pairs over a lossy
     in-memory writer), GPU work through libqfec.so.

Only where /root/reference exists (this container); the built .so travels to
the GPU box with the tree (git-ignored, not gpurun-ignored) for the
end-to-end GPU test (tests/test_integration.py).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.environ.get("QFEC_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "_build")
SRC = os.path.join(OUT, "src")
CORE = os.path.join(SRC, "net", "quic", "core")
PATCH = os.path.join(HERE, "libquic_fec.patch")
LIB = os.path.join(OUT, "libquic_fec_patched.so")
# the same objects linked against tests/cpp/cpu_qfec_stub.c (a CPU restatement
# of the qfec entry points the host code calls) instead of libqfec.so: TEST
# INFRASTRUCTURE, so the connection path's FEC (groups, arena, zero-copy
# capture, revival, acks) runs in the CPU suite; never loaded by the product
LIB_CPU = os.path.join(OUT, "libquic_fec_patched_cpustub.so")
STUB = os.path.join(ROOT, "tests", "cpp", "cpu_qfec_stub.c")

PATCHED = ["quic_protocol.h", "quic_protocol.cc", "quic_framer.h", "quic_framer.cc",
           "quic_connection_stats.h", "quic_connection_stats.cc",
           "quic_packet_creator.h", "quic_packet_creator.cc", "quic_packet_generator.h",
           "quic_connection.h", "quic_connection.cc", "quic_received_packet_manager.h",
           "quic_received_packet_manager.cc", "quic_sent_packet_manager.h",
           "quic_sent_packet_manager.cc"]
FEC_HOST = ["quic_fec_group.h", "quic_fec_group.cc", "quic_fec_wire.h", "quic_fec_wire.cc",
            "quic_fec_connection.h", "quic_fec_connection.cc"]
# translation units syntax-checked against the reference headers
SYNTAX_UNITS = ["quic_protocol.cc", "quic_framer.cc", "quic_packet_creator.cc",
                "quic_connection.cc", "quic_received_packet_manager.cc",
                "quic_sent_packet_manager.cc", "quic_fec_group.cc", "quic_fec_wire.cc",
                "quic_fec_connection.cc"]
# linked: the patched units + the FEC host code (from _build) and, unmodified
# from the reference tree, what the framer and the packet creator reach
LINK_PATCHED = ["quic_protocol.cc", "quic_framer.cc", "quic_packet_creator.cc",
                "quic_connection.cc", "quic_connection_stats.cc",
                "quic_received_packet_manager.cc", "quic_sent_packet_manager.cc",
                "quic_fec_group.cc", "quic_fec_wire.cc", "quic_fec_connection.cc"]
LINK_REF = [
    "net/quic/core/crypto/quic_decrypter.cc", "net/quic/core/crypto/quic_encrypter.cc",
    "net/quic/core/quic_flags.cc", "net/quic/core/quic_data_reader.cc",
    "net/quic/core/quic_data_writer.cc", "net/quic/core/quic_utils.cc",
    "net/quic/core/crypto/crypto_framer.cc", "net/quic/core/crypto/crypto_handshake_message.cc",
    "net/quic/core/quic_socket_address_coder.cc", "net/base/ip_endpoint.cc",
    "net/base/ip_address.cc", "net/quic/core/crypto/null_encrypter.cc",
    "net/quic/core/crypto/null_decrypter.cc", "net/quic/core/crypto/aes_128_gcm_12_encrypter.cc",
    "net/quic/core/crypto/aes_128_gcm_12_decrypter.cc",
    "net/quic/core/crypto/chacha20_poly1305_encrypter.cc",
    "net/quic/core/crypto/chacha20_poly1305_decrypter.cc",
    "net/quic/core/crypto/aead_base_encrypter.cc", "net/quic/core/crypto/aead_base_decrypter.cc",
    "net/quic/core/crypto/scoped_evp_aead_ctx.cc", "net/quic/core/crypto/quic_random.cc",
    "net/quic/core/quic_simple_buffer_allocator.cc", "net/base/int128.cc", "crypto/hkdf.cc",
    "crypto/hmac.cc", "crypto/random.cc", "base/logging.cc", "base/debug/alias.cc",
    "base/debug/debugger.cc", "base/debug/stack_trace.cc", "base/debug/activity_tracker.cc",
    "base/synchronization/lock.cc", "base/synchronization/lock_impl_posix.cc",
    "base/threading/platform_thread_posix.cc", "base/threading/platform_thread_linux.cc",
    "base/threading/thread_checker_impl.cc", "base/threading/thread_local_storage.cc",
    "base/threading/thread_local_storage_posix.cc", "base/threading/thread_local_posix.cc",
    "base/strings/string_piece.cc", "base/time/time.cc", "base/time/time_posix.cc",
    "base/sequence_token.cc", "base/lazy_instance.cc", "base/at_exit.cc",
    "base/callback_internal.cc", "base/vlog.cc", "base/strings/stringprintf.cc",
    "base/strings/string_number_conversions.cc", "base/memory/singleton.cc", "base/rand_util.cc",
    "base/rand_util_posix.cc",
    # what the patched QuicConnection reaches (quic_connection.cc: packet
    # generator, sent / received packet managers, congestion control, config,
    # UMA histograms), found by linking with -z defs until nothing is missing
    "net/quic/core/quic_alarm.cc", "net/quic/core/quic_bandwidth.cc",
    "net/quic/core/quic_clock.cc", "net/quic/core/quic_types.cc",
    "net/quic/core/quic_packet_generator.cc", "net/quic/core/quic_sent_entropy_manager.cc",
    "net/quic/core/quic_multipath_sent_packet_manager.cc",
    "net/quic/core/quic_unacked_packet_map.cc", "net/quic/core/quic_time.cc",
    "net/quic/core/quic_sustained_bandwidth_recorder.cc", "net/quic/core/quic_config.cc",
    "net/quic/core/congestion_control/general_loss_algorithm.cc",
    "net/quic/core/congestion_control/pacing_sender.cc",
    "net/quic/core/congestion_control/rtt_stats.cc",
    "net/quic/core/congestion_control/send_algorithm_interface.cc",
    "net/quic/core/congestion_control/cubic.cc", "net/quic/core/congestion_control/cubic_bytes.cc",
    "net/quic/core/congestion_control/hybrid_slow_start.cc",
    "net/quic/core/congestion_control/prr_sender.cc",
    "net/quic/core/congestion_control/tcp_cubic_sender_base.cc",
    "net/quic/core/congestion_control/tcp_cubic_sender_bytes.cc",
    "net/quic/core/congestion_control/tcp_cubic_sender_packets.cc",
    "net/base/address_family.cc", "net/base/net_errors.cc", "base/metrics/histogram.cc",
    "base/metrics/histogram_base.cc", "base/metrics/bucket_ranges.cc",
    "base/metrics/histogram_samples.cc", "base/metrics/sample_vector.cc",
    "base/metrics/statistics_recorder.cc", "base/metrics/metrics_hashes.cc",
    "base/metrics/persistent_histogram_allocator.cc",
    "base/metrics/persistent_memory_allocator.cc", "base/metrics/persistent_sample_map.cc",
    "base/metrics/sample_map.cc", "base/metrics/sparse_histogram.cc", "base/values.cc",
    "base/md5.cc", "base/pickle.cc", "base/posix/safe_strerror.cc", "base/strings/string16.cc",
    "base/strings/utf_string_conversions.cc", "base/strings/string_util.cc",
    "base/strings/utf_string_conversion_utils.cc", "base/third_party/icu/icu_utf.cc"]
LINK_BSSL = [
    "crypto/cipher/aead.c", "crypto/cipher/e_aes.c", "crypto/cipher/e_chacha20poly1305.c",
    "crypto/err/err.c", "crypto/mem.c", "crypto/crypto.c", "crypto/cpu-intel.c",
    "crypto/thread_pthread.c", "crypto/aes/aes.c", "crypto/modes/gcm.c", "crypto/modes/ctr.c",
    "crypto/chacha/chacha.c", "crypto/poly1305/poly1305.c", "crypto/poly1305/poly1305_vec.c",
    "crypto/hkdf/hkdf.c", "crypto/hmac/hmac.c", "crypto/digest/digest.c",
    "crypto/digest/digests.c", "crypto/sha/sha1.c", "crypto/sha/sha256.c", "crypto/sha/sha512.c",
    "crypto/md4/md4.c", "crypto/md5/md5.c", "crypto/rand/rand.c", "crypto/rand/urandom.c"]

# hidden visibility: only the shim's C API leaves the library, so nothing in it
# can bind to (or be interposed by) the standalone net:: mirror libqfec.so exports
CXXFLAGS = ["-std=gnu++11", "-O2", "-DNDEBUG", "-w", "-fPIC", "-ffunction-sections",
            "-fdata-sections", "-fvisibility=hidden", "-fvisibility-inlines-hidden",
            "-DQFEC_WITH_LIBQUIC"]


def _incs():
    return ["-I", SRC, "-I", os.path.join(REF, "src"), "-I",
            os.path.join(REF, "boringssl", "include"), "-I", os.path.join(ROOT, "include"),
            "-I", os.path.join(REF, "src", "third_party", "protobuf", "src")]


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "src", "net", "quic", "core"))


def prepare() -> None:
    """Fresh copy of the originals, the patch applied, the FEC host code in."""
    if os.path.isdir(SRC):
        shutil.rmtree(SRC)
    os.makedirs(CORE)
    for f in PATCHED:
        shutil.copy(os.path.join(REF, "src", "net", "quic", "core", f), CORE)
    subprocess.run(["patch", "-p1", "-s", "--no-backup-if-mismatch", "-i", PATCH], cwd=OUT,
                   check=True)
    for f in FEC_HOST:
        shutil.copy(os.path.join(ROOT, "libquic_amd", "csrc", f), CORE)


def syntax_check() -> list:
    """(unit, returncode, stderr) for every unit; all must be 0."""
    def one(u):
        r = subprocess.run(["g++", *CXXFLAGS, "-fsyntax-only", *_incs(), os.path.join(CORE, u)],
                           capture_output=True, text=True)
        return u, r.returncode, r.stderr
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(one, SYNTAX_UNITS))


def _inputs_mtime():
    """Newest of what every unit may include beyond its own source: the patch
    (it changes reference headers, e.g. QuicAckFrame's layout) and the FEC
    host headers."""
    hs = [PATCH] + [os.path.join(ROOT, "libquic_amd", "csrc", f) for f in FEC_HOST
                    if f.endswith(".h")] + [os.path.join(ROOT, "include", "qfec.h")]
    return max(os.path.getmtime(h) for h in hs)


def _obj(src, flags, name, always=False):
    o = os.path.join(OUT, "obj", name + ".o")
    if (always or not os.path.exists(o) or
            os.path.getmtime(o) < max(os.path.getmtime(src), _inputs_mtime())):
        os.makedirs(os.path.dirname(o), exist_ok=True)
        subprocess.run([*flags, "-c", src, "-o", o], check=True)
    return o


def build_lib() -> str:
    cc = ["gcc", "-std=gnu11", "-O2", "-DNDEBUG", "-w", "-fPIC", "-D_GNU_SOURCE", "-fvisibility=hidden",
          "-DOPENSSL_NO_ASM", "-ffunction-sections", "-fdata-sections", "-I",
          os.path.join(REF, "boringssl", "include")]
    cxx = ["g++", *CXXFLAGS, *_incs()]
    jobs = [(os.path.join(CORE, u), cxx, "patched_" + u.replace("/", "_")) for u in LINK_PATCHED]
    jobs += [(os.path.join(REF, "src", u), cxx, "ref_" + u.replace("/", "_")) for u in LINK_REF]
    jobs += [(os.path.join(REF, "boringssl", u), cc, "bssl_" + u.replace("/", "_"))
             for u in LINK_BSSL]
    # the shims include the patched headers (fresh copies every build)
    jobs += [(os.path.join(HERE, "patched_shim.cc"), cxx, "patched_shim", True),
             (os.path.join(HERE, "connection_shim.cc"), cxx, "connection_shim", True)]
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(lambda j: _obj(*j), jobs))
    libdir = os.path.join(ROOT, "libquic_amd")
    subprocess.run(["g++", "-shared", "-pthread", "-Wl,--gc-sections", "-Wl,-z,defs", "-Wl,-Bsymbolic",
                    "-o", LIB + ".tmp", *objs, "-L", libdir, "-lqfec",
                    "-Wl,-rpath,$ORIGIN/../../libquic_amd", "-Wl,-rpath-link,/opt/rocm/lib"],
                   check=True)
    os.replace(LIB + ".tmp", LIB)
    stub = _obj(STUB, ["gcc", "-std=c11", "-O2", "-fPIC", "-fvisibility=hidden", "-I",
                       os.path.join(ROOT, "include")], "cpu_qfec_stub")
    subprocess.run(["g++", "-shared", "-pthread", "-Wl,--gc-sections", "-Wl,-z,defs", "-Wl,-Bsymbolic",
                    "-o", LIB_CPU + ".tmp", *objs, stub], check=True)
    os.replace(LIB_CPU + ".tmp", LIB_CPU)
    return LIB


def regen_patch() -> str:
    """Maintainer step: rewrite integration/libquic_fec.patch from the edited
    copies under _build/src (after prepare() and edits there), one
    `diff -u` per PATCHED file against /root/reference, in file name order."""
    out = []
    for f in sorted(PATCHED):
        rel = f"src/net/quic/core/{f}"
        r = subprocess.run(["diff", "-u", "--label", "a/" + rel, "--label", "b/" + rel,
                            os.path.join(REF, rel), os.path.join(CORE, f)],
                           capture_output=True, text=True)
        if r.returncode == 0:
            continue
        if r.returncode != 1:
            raise RuntimeError(r.stderr)
        out.append(f"diff --git a/{rel} b/{rel}\n" + r.stdout)
    text = "".join(out)
    with open(PATCH, "w") as fh:
        fh.write(text)
    return PATCH


def build() -> bool:
    """prepare + syntax check + link; False where the reference is absent."""
    if not available():
        return False
    prepare()
    bad = [(u, e) for u, rc, e in syntax_check() if rc != 0]
    if bad:
        raise RuntimeError("patched libquic does not compile:\n" +
                           "\n".join(f"{u}:\n{e[-3000:]}" for u, e in bad))
    build_lib()
    return True


if __name__ == "__main__":
    if "--regen-patch" in sys.argv:
        print("rewrote", regen_patch())
        sys.exit(0)
    ok = build()
    print("integration build:", "ok" if ok else "skipped (no /root/reference)")
    sys.exit(0)
