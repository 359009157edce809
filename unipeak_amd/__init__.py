"""unipeak_amd -- MI355X-native KDE smoothing + enriched-region scan.

The product is the C-ABI library ``unipeak_amd/lib/libunipeak_hip.so``
(include/unipeak_hip.h) and the C++ CLIs in ``bin/``.  This package only
exposes a ctypes binding of that library (``unipeak_amd.capi``) for the
tests and bench.py; there is no Python or CPU fallback: if the HIP library
is missing, loading it raises.
"""
from .capi import Lib, UpError, Region, load_library  # noqa: F401

__version__ = "1.0"
