"""MI355X-native Shadow network plane: routing table + per-round packet hand-off.

The product is libshdnet.so (include/shdnet.h: host C + hand-written HIP
kernels for gfx950).  This package is its Python host mirror (ctypes) plus the
seeded synthetic workloads used by tests and bench.py.
"""
from . import scenario, synth  # noqa: F401
from ._lib import ShdError  # noqa: F401
from .topology import Topology  # noqa: F401

__all__ = ["Topology", "ShdError", "scenario", "synth"]
