"""murr_amd — MI355X-native row-blob codec for murr's `src/io` encode/decode path.

Product code: libmurr_codec.so (HIP kernels for gfx950 + C ABI, include/murr_codec.h)
and this thin host mirror of the reference interface (Table / Store /
ReadBatchBuilder / SegmentSchema).  There is no CPU fallback: every compute call
goes through the HIP library and raises if it cannot be loaded.
"""
from . import _abi
from .errors import (ArrowError, DeviceError, IoError, MurrError, SegmentError, TableAlreadyExists,
                     TableError, TableNotFound)
from .schema import ColumnSchema, DTypeName, SegmentColumnSchema, SegmentSchema, TableSchema, dtype_from_arrow

__all__ = ["ArrowError", "DeviceError", "IoError", "MurrError", "SegmentError", "TableAlreadyExists",
           "TableError", "TableNotFound", "ColumnSchema", "DTypeName", "SegmentColumnSchema",
           "SegmentSchema", "TableSchema", "dtype_from_arrow", "lib"]


def lib():
    """The loaded libmurr_codec.so (raises ImportError when it is not built)."""
    return _abi.lib()
