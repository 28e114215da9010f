"""4c_amd -- MI355X-native SOLID element evaluation + global assembly for 4C.

The product is libfourc_gpu.so (4c_amd/csrc, C ABI in include/fourc_gpu.h).  This package only
loads it; `import importlib; fcg = importlib.import_module("4c_amd").fcg`.
"""
from . import fcg  # noqa: F401

__all__ = ["fcg"]
