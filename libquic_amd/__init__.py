"""libquic_amd — MI355X-native QUIC forward-error-correction (XOR parity) path.

The product is native: ``libqfec.so`` (gfx950 HIP kernels + the C-ABI declared
in include/qfec.h + the C++ QuicFecGroup host mirror).  ``libquic_amd.qfec`` is a
thin ctypes binding used by tests and bench.py.  There is no CPU fallback.
"""
from . import qfec  # noqa: F401

__all__ = ["qfec"]
