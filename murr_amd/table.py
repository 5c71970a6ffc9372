"""Table (src/io/table/mod.rs:20-155): the caller of both directions.

`write` keeps the reference's validation (canonical projection, Utf8 non-null
key, per-column dtype check = make_decoder's downcast) and replaces the serial
per-row WriteRow loop with one GPU encode (murr_encode_host: pinned H2D ->
encode kernel -> D2H).  `read` resolves the requested names and hands a
GPU-batched ReadBatchBuilder down to the store (table/mod.rs:114-129).
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np
import pyarrow as pa

from . import _abi
from .errors import ArrowError, SegmentError, TableError, raise_status
from .row import IpcReadBatchBuilder, ReadBatchBuilder, default_context
from .schema import DTypeName, SegmentSchema, TableSchema
from .store import KeyValue, Store


class Table:
    def __init__(self, store: Store, name: str, table: TableSchema, ctx=None):
        """Table::build (table/mod.rs:131-154)."""
        key_col = table.columns.get(table.key)
        if key_col is None:
            raise TableError(f"key column '{table.key}' not in schema")
        if key_col.dtype != DTypeName.Utf8:
            raise TableError("io currently supports Utf8 keys only")
        self.store = store
        self.name = name
        self.table = table
        self.segment = SegmentSchema.from_table(table)
        self.columns = {c.name: i for i, c in enumerate(self.segment.columns)}
        self._ctx = ctx
        self.lock = threading.RLock()  # stands in for Arc<RwLock<S>>

    @property
    def ctx(self):
        """The device context, created on first compute call (host-only
        validation paths never touch the GPU)."""
        if self._ctx is None:
            self._ctx = default_context()
        return self._ctx

    def prepare(self):
        """Compile (or load from the code-object cache) the layout's decode and
        encode kernels now (murr_segment_prepare), so no read or write pays
        for it: the decode kernel is specialised on the segment layout only,
        and every projection a read asks for runs the same code object."""
        from .errors import raise_status
        if not getattr(self, "_prepared", False):
            raise_status(self.ctx.L.murr_segment_prepare(self.ctx.h, C.byref(self.segment.c)),
                         what="murr_segment_prepare")
            self._prepared = True

    @classmethod
    def create(cls, store: Store, name: str, table: TableSchema, ctx=None) -> "Table":
        store.create_table(name, table)
        return cls(store, name, table, ctx)

    @classmethod
    def open(cls, store: Store, name: str, table: TableSchema, ctx=None) -> "Table":
        return cls(store, name, table, ctx)

    def schema(self) -> TableSchema:
        return self.table

    # -- write ------------------------------------------------------------------
    def validate(self, batch: pa.RecordBatch):
        """Table::write's checks (table/mod.rs:54-96): canonical projection,
        Utf8 non-null key, make_decoder's dtype downcast per column
        (src/io/codec/mod.rs:78-85).  Returns (key array, arrays in segment
        order)."""
        canonical = self.table.to_arrow()
        names = batch.schema.names
        indices = []
        for f in canonical:
            if f.name not in names:
                raise ArrowError(f"Schema error: Unable to get field named \"{f.name}\". "
                                 f"Valid fields: {names}")
            indices.append(names.index(f.name))
        ordered = batch.select(indices)
        key_idx = canonical.get_field_index(self.table.key)
        key_array = ordered.column(key_idx)
        if key_array.type != pa.string():
            raise SegmentError(f"key column '{self.table.key}' must be Utf8")
        if key_array.null_count > 0:
            raise SegmentError("null in key column")
        arrays = []
        for col in self.segment.columns:
            arr = ordered.column(canonical.get_field_index(col.name))
            want = col.dtype.arrow_dtype()
            if arr.type != want:
                raise SegmentError(f"expected {want}, got {arr.type}")
            arrays.append(arr)
        return key_array, arrays

    def encode(self, batch: pa.RecordBatch):
        """Table::write up to the store call: returns (keys StringArray, blob
        uint8 ndarray, row_off uint64 ndarray)."""
        key_array, arrays = self.validate(batch)
        n = batch.num_rows
        seg = self.segment
        hcols = (_abi.HostColIn * max(len(seg), 1))()
        keep = []
        for i, col in enumerate(seg.columns):
            arr = arrays[i]
            bufs = arr.buffers()
            keep.append(bufs)
            hc = hcols[i]
            hc.col.offset = arr.offset
            hc.col.validity = bufs[0].address if (bufs[0] is not None and arr.null_count) else None
            if col.dtype == DTypeName.Utf8:
                hc.col.offsets = bufs[1].address
                hc.col.values = bufs[2].address if bufs[2] is not None and bufs[2].size else None
                hc.values_bytes = bufs[2].size if bufs[2] is not None else 0
                if not hc.col.values:
                    pad = np.zeros(16, np.uint8)
                    keep.append(pad)
                    hc.col.values = pad.ctypes.data
                    hc.values_bytes = 16
            else:
                hc.col.values = bufs[1].address
                hc.values_bytes = bufs[1].size
        blob = C.POINTER(C.c_uint8)()
        row_off = C.POINTER(C.c_uint64)()
        blen = C.c_uint64()
        err = _abi.Error()
        st = self.ctx.L.murr_encode_host(self.ctx.h, C.byref(seg.c), hcols, n, C.byref(blob),
                                         C.byref(blen), C.byref(row_off), C.byref(err))
        raise_status(st, err, "Table::write encode")
        try:
            out = np.frombuffer(C.string_at(blob, blen.value), dtype=np.uint8).copy() if blen.value \
                else np.zeros(0, np.uint8)
            offs = np.frombuffer(C.string_at(row_off, (n + 1) * 8), dtype=np.uint64).copy()
        finally:
            self.ctx.L.murr_host_free(self.ctx.h, blob)
            self.ctx.L.murr_host_free(self.ctx.h, row_off)
        return key_array, out, offs

    def write(self, batch: pa.RecordBatch):
        """Table::write (table/mod.rs:54-112)."""
        keys, blob, offs = self.encode(batch)
        raw = blob.tobytes()
        kv = (KeyValue(keys[i].as_py().encode(), raw[offs[i]:offs[i + 1]]) for i in range(len(keys)))
        with self.lock:
            self.store.write(self.name, kv)

    # -- read -------------------------------------------------------------------
    def read(self, keys, columns) -> pa.RecordBatch:
        """Table::read (table/mod.rs:114-129)."""
        req = []
        for name in columns:
            idx = self.columns.get(name)
            if idx is None:
                raise SegmentError(f"column '{name}' not found")
            req.append(self.segment.columns[idx])
        builder = ReadBatchBuilder(self.segment, req, len(keys), self.ctx)
        key_bytes = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
        with self.lock:
            return self.store.read(self.name, key_bytes, builder)

    def read_ipc(self, keys, columns, alignment: int = 64) -> bytes:
        """Table::read + the HTTP handler's StreamWriter (handlers.rs:88-101):
        the read as an Arrow IPC stream (arrow-rs default alignment 64)."""
        req = []
        for name in columns:
            idx = self.columns.get(name)
            if idx is None:
                raise SegmentError(f"column '{name}' not found")
            req.append(self.segment.columns[idx])
        builder = IpcReadBatchBuilder(self.segment, req, len(keys), self.ctx, alignment)
        key_bytes = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
        with self.lock:
            return self.store.read(self.name, key_bytes, builder)
