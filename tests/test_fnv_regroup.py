"""CPU check of the three-bytes-per-multiply FNV-1a-128 step (fnv_step3 in
libquic_amd/csrc/qpp_kernels.hip) against the byte-serial recurrence of the
reference (quic_utils.cc:31-54): tools/tune/fnv_r3_check.c restates the device
function in C, compiles with gcc and compares 4M random triples (edge states
with tiny low limbs included) and a 3.2 MB stream hashed in 16-byte chunks.
The GPU tests check the kernels themselves (test_hip_protect.py)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_fnv_step3_matches_byte_serial(tmp_path):
    exe = os.path.join(str(tmp_path), "fnv_r3_check")
    src = os.path.join(ROOT, "tools", "tune", "fnv_r3_check.c")
    subprocess.run(["gcc", "-O2", "-o", exe, src], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    assert " 0 mismatches" in out, out
