"""Connection-level FEC (libquic_amd/csrc/quic_fec_connection.h): the C++ test
binary tests/cpp/test_quic_fec_connection.  CPU: group bookkeeping of the send
and receive sides (nothing is flushed, no device).  GPU: a lossy, reordering
multi-connection simulation whose closed groups and revivable groups are
flushed in one ragged launch per tick, revived packets checked bit-exactly."""
import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_quic_fec_connection")


def _exe():
    if not os.path.exists(EXE):
        from libquic_amd import build as B
        B.build_cpp_tests()
    return EXE


def test_connection_bookkeeping_cpu():
    r = subprocess.run([_exe(), "--cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.gpu
def test_connection_simulation_gpu():
    r = subprocess.run([_exe()], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    sims = [l for l in r.stdout.splitlines() if l.startswith("simulation:")]
    assert len(sims) == 2
    for l in sims:
        revived = int(l.split(" revived (")[0].split(", ")[-1])
        assert revived > 0, l
