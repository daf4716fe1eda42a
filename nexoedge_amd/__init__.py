"""nexoedge_amd -- MI355X-native Reed-Solomon coding path for Nexoedge.

The product is libnxec.so (C ABI: include/nxec.h; C++ RSCode surface:
nexoedge_amd/csrc/coding/).  This package only loads it and offers a thin
Python view for tests and benchmarks.  Import fails if the library is not
built: there is no CPU fallback.
"""
from ._lib import LIB_PATH, NxecError, lib  # noqa: F401  (raises ImportError when unbuilt)
from . import nxec  # noqa: F401

__version__ = lib.nxec_version().decode()
