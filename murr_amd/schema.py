"""Schema types: DTypeName / ColumnSchema / TableSchema (src/core/schema.rs) and
the row layout SegmentSchema / SegmentColumnSchema (src/io/schema.rs).

The layout arithmetic is done by the C ABI (murr_segment_init), so the Python
side cannot drift from the kernels' view of a row.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass, field

import pyarrow as pa

from . import _abi
from .errors import MurrError, SegmentError


class DTypeName(enum.IntEnum):
    """src/core/schema.rs:6-19, same members and order (serde lowercase names)."""
    Utf8 = 0
    Bool = 1
    Int8 = 2
    Int16 = 3
    Int32 = 4
    Int64 = 5
    UInt8 = 6
    UInt16 = 7
    UInt32 = 8
    UInt64 = 9
    Float32 = 10
    Float64 = 11

    @property
    def serde_name(self) -> str:
        return self.name.lower()

    @classmethod
    def parse(cls, v) -> "DTypeName":
        if isinstance(v, DTypeName):
            return v
        if isinstance(v, int):
            return cls(v)
        for m in cls:
            if m.serde_name == str(v).lower():
                return m
        raise MurrError(f"unknown dtype {v!r}")

    def size(self) -> int:
        """DType::size (src/io/codec/<dtype>.rs)."""
        return _abi.lib().murr_dtype_size(int(self))

    def arrow_dtype(self) -> pa.DataType:
        """DType::arrow_dtype."""
        return _ARROW[self]


_ARROW = {
    DTypeName.Utf8: pa.string(), DTypeName.Bool: pa.bool_(), DTypeName.Int8: pa.int8(),
    DTypeName.Int16: pa.int16(), DTypeName.Int32: pa.int32(), DTypeName.Int64: pa.int64(),
    DTypeName.UInt8: pa.uint8(), DTypeName.UInt16: pa.uint16(), DTypeName.UInt32: pa.uint32(),
    DTypeName.UInt64: pa.uint64(), DTypeName.Float32: pa.float32(), DTypeName.Float64: pa.float64(),
}


def dtype_from_arrow(dt: pa.DataType) -> DTypeName:
    """TryFrom<&DataType> for DTypeName (src/io/schema.rs:70-91)."""
    for k, v in _ARROW.items():
        if v == dt:
            return k
    raise SegmentError(f"unsupported dtype {dt}")


@dataclass
class ColumnSchema:
    """src/core/schema.rs:21-33 (nullable defaults to true)."""
    dtype: DTypeName
    nullable: bool = True

    def __post_init__(self):
        self.dtype = DTypeName.parse(self.dtype)


@dataclass
class TableSchema:
    """src/core/schema.rs:35-39: key column name + IndexMap of columns (insertion order)."""
    key: str
    columns: dict = field(default_factory=dict)  # name -> ColumnSchema, insertion-ordered

    def to_arrow(self) -> pa.Schema:
        """From<&TableSchema> for Schema (src/io/schema.rs:56-68)."""
        fields = [pa.field(n, c.dtype.arrow_dtype(), c.nullable) for n, c in self.columns.items()]
        return pa.schema(fields, metadata={"key": self.key})


@dataclass(frozen=True)
class SegmentColumnSchema:
    """src/io/schema.rs:8-14."""
    index: int
    dtype: DTypeName
    name: str
    offset: int


class SegmentSchema:
    """src/io/schema.rs:16-54: non-key columns in TableSchema order; bit index =
    position, offset = running sum of sizes; capacity = sum; bitset = ceil(n/8)."""

    def __init__(self, columns):
        """SegmentSchema::new over (name, dtype) pairs or SegmentColumnSchema."""
        names, dtypes = [], []
        for c in columns:
            if isinstance(c, SegmentColumnSchema):
                names.append(c.name)
                dtypes.append(c.dtype)
            else:
                names.append(c[0])
                dtypes.append(DTypeName.parse(c[1]))
        n = len(dtypes)
        self._dt = (C.c_uint32 * max(n, 1))(*[int(d) for d in dtypes])
        self._cols = (_abi.Column * max(n, 1))()
        self.c = _abi.Segment()
        st = _abi.lib().murr_segment_init(self._dt, n, self._cols, C.byref(self.c))
        if st:
            raise SegmentError(f"segment layout: {_abi.status_str(st)}")
        self.columns = [SegmentColumnSchema(self._cols[i].index, dtypes[i], names[i],
                                            self._cols[i].offset) for i in range(n)]

    @classmethod
    def from_table(cls, schema: TableSchema) -> "SegmentSchema":
        return cls([(n, c.dtype) for n, c in schema.columns.items() if n != schema.key])

    @property
    def capacity(self) -> int:
        return self.c.capacity

    @property
    def bitset_size(self) -> int:
        return self.c.bitset_size

    def __len__(self):
        return len(self.columns)
