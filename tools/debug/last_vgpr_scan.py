"""CLI over libquic_amd/isa_guard.py (the last-VGPR 64-bit shift scan) for
experiment builds: python tools/debug/last_vgpr_scan.py file.{s,so,co} [...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from libquic_amd import isa_guard  # noqa: E402

if __name__ == "__main__":
    sys.argv[0] = "last_vgpr_scan"
    isa_guard.main(sys.argv[1:])
