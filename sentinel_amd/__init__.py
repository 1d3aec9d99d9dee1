"""MI355X-native admission engine for Sentinel's statistics-and-decision path.

The decisions are computed by hand-written HIP kernels for gfx950 in
libsentinel_amd.so (C-ABI: include/sentinel_amd.h).  This package is the
host-side mirror of the reference's Java interface for that path.
"""
from ._lib import EngineError, LIB_PATH  # noqa: F401

__all__ = ["EngineError", "LIB_PATH"]
