"""The installed libqfec.so has no 64-bit VALU shift reading its amount from
the wave's last allocated VGPR: on gfx950 such a shift uses v0's value instead
in a fraction of executions when several waves share a SIMD — the cause of
the round-1 ragged build's wrong parity (DESIGN.md §4,
tools/debug/last_vgpr_ops.hip).  build.build_lib() refuses to install such a
library; this checks the one in the tree, and that the scan finds the
pattern where it is (an assembly snippet with the round-1 instruction)."""
import os

from libquic_amd import isa_guard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "libquic_amd", "libqfec.so")


def test_product_library_has_no_last_vgpr_shift_amount():
    assert os.path.exists(LIB), "build() first"
    kernels = list(isa_guard.kernels(LIB))
    assert len(kernels) > 20  # every FEC / protection / entropy kernel was read
    assert isa_guard.scan(LIB) == []


def test_scan_flags_the_round1_pattern(tmp_path):
    s = tmp_path / "k.s"
    s.write_text(
        "_Zbad:\n"
        "\tv_bitop3_b32 v55, v54, 63, 56 bitop3:0x6c\n"
        "\tv_lshlrev_b64 v[22:23], v55, v[22:23]\n"
        ".Lfunc_end0:\n"
        "_Zgood:\n"
        "\tv_lshlrev_b64 v[22:23], v40, v[22:23]\n"
        "\tv_lshlrev_b64 v[22:23], v68, v[22:23]\n"  # 69 VGPRs -> 72 allocated: v71 is last
        ".Lfunc_end1:\n"
        "\t.amdhsa_kernel _Zbad\n\t\t.amdhsa_next_free_vgpr 56\n\t.end_amdhsa_kernel\n"
        "\t.amdhsa_kernel _Zgood\n\t\t.amdhsa_next_free_vgpr 69\n\t.end_amdhsa_kernel\n")
    hits = isa_guard.scan(str(s))
    assert [h[0] for h in hits] == ["_Zbad"]


def test_product_kernels_use_no_scratch():
    """no kernel of libqfec.so spills to scratch (private segment 0 bytes)"""
    segs = isa_guard.private_segments(LIB)
    assert len(segs) == len(list(isa_guard.kernels(LIB)))
    assert {k: v for k, v in segs.items() if v} == {}
