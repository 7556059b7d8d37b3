"""fbthrift_amd — MI355X-native bulk Thrift record codec.

Binary and Compact protocol encode/decode of whole batches of same-schema
records on gfx950, byte-identical to fbthrift's CPU protocols. The product is
the C-ABI library fbthrift_amd/lib/libtgpu.so (include/thrift_gpu.h) and its
C++ host mirror (include/thrift_gpu/GpuBatchSerializer.h); this Python package
is the host mirror used by tests and bench.py.
"""
from . import _lib  # noqa: F401
from ._lib import PROTOCOL_BINARY, PROTOCOL_COMPACT  # noqa: F401
from .schema import Field, Schema, Struct  # noqa: F401

__all__ = ["Field", "Schema", "Struct", "PROTOCOL_BINARY", "PROTOCOL_COMPACT"]
