"""redpanda_amd — MI355X-native record-batch validation / decode engine.

The product is the HIP library librpgpu.so behind the C ABI in
include/rpgpu.h.  This package holds its sources (csrc/), the ctypes view of
that ABI (abi.py), the engine wrapper (engine.py), the partition shard and
summary gather (shard.py) and the build recipe (_build.py).
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
