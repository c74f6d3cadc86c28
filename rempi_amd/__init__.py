"""rempi_amd -- MI355X-native Clock Delta Compression (CDC) for ReMPI record/replay.

The codec itself is libcdcx.so (HIP kernels for gfx950 behind the C ABI of
include/cdcx.h).  This package holds the ctypes binding (cdcx.py), the sharding helpers of
the many-rank bench (shard.py) and the command-line tools over the C ABI (replay.py,
transcode.py).
"""
from .cdcx import CdcxError, Context, GenParams, default_gen_params, generate_host, lib  # noqa: F401

__all__ = ["CdcxError", "Context", "GenParams", "default_gen_params", "generate_host", "lib"]
