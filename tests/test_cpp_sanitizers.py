"""The host C++ under sanitizers on the CPU.

tests/cpp/test_quic_fec_group.cc and test_quic_fec_connection.cc — the
payload arena (per-thread slabs, atomic release, the process-wide pool of a
finished thread's slabs), QuicFecGroup bookkeeping, the ragged CSR builders,
QuicFecReceiver's group map, the encode / revive batches — built with
AddressSanitizer + UBSan (arena slabs poisoned outside live payloads) and the
group test with ThreadSanitizer, against tests/cpp/cpu_qfec_stub.c, a CPU
restatement of the five C-ABI calls the host code makes (test infrastructure,
never part of libqfec.so).  No GPU.
"""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def binaries():
    from libquic_amd import build as B
    return B.build_cpp_sanitized()


@pytest.mark.parametrize("name", ["san_test_quic_fec_group", "san_test_quic_fec_connection",
                                  "tsan_test_quic_fec_group", "san_test_layout_guard"])
def test_host_cpp_under_sanitizers(binaries, name):
    exe = os.path.join(ROOT, "tests", "cpp", "build", name)
    assert exe in binaries
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert " 0 failures" in out, out[-2000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    if name == "san_test_layout_guard":
        # a caller built against another quic_fec_group.h
        # is refused loudly, and nothing is written (ASan clean above)
        assert "refused (QUIC_INTERNAL_ERROR)" in out, out[-2000:]
