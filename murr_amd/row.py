"""ReadBatchBuilder (src/io/row/read.rs:62-110), batched on the GPU.

The store feeds rows exactly as in the reference (`add_row` / `add_empty` in
caller order, src/io/store/memory.rs:38-43); rows are copied into a pinned host
staging block by the C ABI, and `build()` runs H2D -> one decode launch -> D2H
and returns a pyarrow RecordBatch whose fields are nullable and in request
order (read.rs:100-109).
"""
from __future__ import annotations

import bisect
import ctypes as C

import numpy as np
import pyarrow as pa

from . import _abi
from .errors import ArrowError, raise_status
from .schema import DTypeName, SegmentColumnSchema, SegmentSchema

_ctx = {}


def default_context(device: int = 0):
    from .device import Context
    if device not in _ctx:
        _ctx[device] = Context(device)
    return _ctx[device]


class ReadBatchBuilder:
    def __init__(self, segment: SegmentSchema, columns, capacity: int, ctx=None):
        """ReadBatchBuilder::new(segment, columns, capacity): one output column per
        requested column, request order, duplicates allowed (read.rs:69-83)."""
        self.segment = segment
        self.columns = list(columns)
        self.ctx = ctx or default_context()
        self.L = self.ctx.L
        proj = [c.index if isinstance(c, SegmentColumnSchema) else int(c) for c in self.columns]
        self._proj = (C.c_uint32 * max(len(proj), 1))(*proj)
        self._nproj = len(proj)
        h = C.c_void_p()
        raise_status(self.L.murr_builder_new(self.ctx.h, C.byref(segment.c), self._proj, self._nproj,
                                             int(capacity), C.byref(h)), what="ReadBatchBuilder::new")
        self.h = h

    def __del__(self):
        try:
            if self.h:
                self.L.murr_builder_free(self.h)
                self.h = None
        except Exception:
            pass

    def add_row(self, raw: bytes):
        raise_status(self.L.murr_builder_add_row(self.h, raw, len(raw)), what="add_row")

    def add_empty(self):
        raise_status(self.L.murr_builder_add_empty(self.h), what="add_empty")

    def add_rows(self, rows):
        """Many rows at once; None = missing key."""
        n = len(rows)
        if not n:
            return
        keep = [r if r is not None else None for r in rows]
        ptrs = (C.c_void_p * n)()
        lens = (C.c_uint64 * n)()
        bufs = []
        for i, r in enumerate(keep):
            if r is None:
                ptrs[i] = None
            else:
                b = C.create_string_buffer(bytes(r), len(r))
                bufs.append(b)
                ptrs[i] = C.addressof(b)
                lens[i] = len(r)
        raise_status(self.L.murr_builder_add_rows(self.h, ptrs, lens, n), what="add_rows")

    def _build_host(self):
        if self._nproj == 0:
            raise ArrowError("Arrow error: must either specify a row count or at least one column")
        outs = (_abi.HostArray * self._nproj)()
        err = _abi.Error()
        raise_status(self.L.murr_builder_build(self.h, outs, C.byref(err)), err, "ReadBatchBuilder::build")
        return outs

    def build(self) -> pa.RecordBatch:
        outs = self._build_host()
        if getattr(self, "_cnames", None) is None:
            self._cnames = c_names(self._schema().names)
        return host_arrays_to_batch(outs, self._nproj, self._cnames)

    def _schema(self) -> pa.Schema:
        """The batch schema: Field(name, arrow dtype, nullable) per requested
        column (read.rs:100-109), built once."""
        if getattr(self, "_arrow_schema", None) is None:
            fields = []
            for col in self.columns:
                seg_col = col if isinstance(col, SegmentColumnSchema) else self.segment.columns[int(col)]
                fields.append(pa.field(seg_col.name, seg_col.dtype.arrow_dtype(), True))
            self._arrow_schema = pa.schema(fields)
        return self._arrow_schema

    def last_timing(self):
        tot, h2d, k, d2h = C.c_double(), C.c_float(), C.c_float(), C.c_float()
        self.L.murr_builder_last_timing(self.h, C.byref(tot), C.byref(h2d), C.byref(k), C.byref(d2h))
        return {"total_ms": tot.value, "h2d_ms": h2d.value, "kernel_ms": k.value, "d2h_ms": d2h.value}


class IpcReadBatchBuilder(ReadBatchBuilder):
    """ReadBatchBuilder whose build() returns the Arrow IPC stream the HTTP
    fetch handler writes with StreamWriter (src/api/http/handlers.rs:93-101):
    schema message, one record-batch message, end-of-stream.  The builder's
    host arrays are framed in place (murr_ipc_batch_host), no pyarrow copy."""

    def __init__(self, segment, columns, capacity, ctx=None, alignment: int = 64):
        super().__init__(segment, columns, capacity, ctx)
        self.alignment = alignment

    def build(self) -> bytes:
        from . import ipc
        outs = self._build_host()
        n = outs[0].length
        cols = [c if isinstance(c, SegmentColumnSchema) else self.segment.columns[int(c)] for c in self.columns]
        return ipc.stream(ipc.schema_message(self.segment, cols, self.alignment),
                          ipc.batch_message_host(self.segment, cols, outs, n, self.alignment))


def _copy(ptr, n) -> pa.Buffer:
    return pa.py_buffer(C.string_at(ptr, n)) if n else pa.py_buffer(b"")


_ARROW_TYPE = {int(d): d.arrow_dtype() for d in DTypeName}
_UTF8 = int(DTypeName.Utf8)


_HOST_ARRAY = np.dtype([("values", np.uint64), ("validity", np.uint64), ("offsets", np.uint64), ("length", np.uint64),
                        ("null_count", np.uint64), ("values_len", np.uint64), ("dtype", np.uint32), ("_pad", np.uint32)])
assert _HOST_ARRAY.itemsize == C.sizeof(_abi.HostArray)


def host_arrays_to_arrow(outs, k: int) -> list:
    """murr_host_array_t[0..k) -> pyarrow Arrays, copied out of the library's
    pinned output region (it is reused by the next read).  The descriptors
    are read as one numpy view; when the arrays' buffers fill most of their
    span (they lie in one region), one copy of the span and zero-copy slices
    of it replace a copy per buffer."""
    if not k:
        return []
    t = np.frombuffer((C.c_char * (k * _HOST_ARRAY.itemsize)).from_address(C.addressof(outs)), _HOST_ARRAY, k)
    vals, valid, offs = t["values"].tolist(), t["validity"].tolist(), t["offsets"].tolist()
    ns, ncs, vlen, dts = t["length"].tolist(), t["null_count"].tolist(), t["values_len"].tolist(), t["dtype"].tolist()
    # (pointer, bytes) of every buffer: validity (nulls only), utf8 offsets, values
    vb = [((n + 7) // 8 if v else 0) for n, v in zip(ns, valid)]
    ob = [((n + 1) * 4 if d == _UTF8 else 0) for n, d in zip(ns, dts)]
    spans = sorted((p, b) for p, b in zip(valid + offs + vals, vb + ob + vlen) if p and b)
    # runs of buffers no more than 4 KiB apart are copied as one span each (a
    # prepared read lays the fixed-size buffers out back to back and each utf8
    # column's bytes in a region of its own, sized for the longest rows)
    runs = []  # [lo, hi]
    for p, b in spans:
        if runs and p <= runs[-1][1] + 4096:
            runs[-1][1] = max(runs[-1][1], p + b)
        else:
            runs.append([p, p + b])
    los = [lo for lo, _ in runs]
    bigs = [pa.py_buffer(C.string_at(lo, hi - lo)) for lo, hi in runs]
    empty = pa.py_buffer(b"")

    def buf(p, b):
        if not (p and b):
            return empty
        j = bisect.bisect_right(los, p) - 1
        return bigs[j].slice(p - los[j], b)

    out = []
    for i in range(k):
        bufs = [buf(valid[i], vb[i]) if valid[i] else None]
        if dts[i] == _UTF8:
            bufs.append(buf(offs[i], ob[i]))
        bufs.append(buf(vals[i], vlen[i]))
        out.append(pa.Array.from_buffers(_ARROW_TYPE[dts[i]], ns[i], bufs, null_count=ncs[i]))
    return out


def host_arrays_to_batch(outs, k: int, names, schema: pa.Schema | None = None) -> pa.RecordBatch:
    """murr_host_array_t[0..k) -> one pyarrow RecordBatch through the Arrow C
    Data Interface (murr_arrow_export: the library copies the bytes out of its
    pinned region into an export it owns; pyarrow imports it in one call).
    `names`: a ctypes array of k c_char_p (built once per column list).
    `schema`: the schema of an earlier batch of the same columns (names and
    dtypes): the export then carries no schema and the array is imported
    against this one (saves the schema's export and parse on every read)."""
    arr = _abi.ArrowArray()
    L = _abi.lib()
    if schema is not None:
        raise_status(L.murr_arrow_export(outs, k, names, C.byref(arr), None), what="murr_arrow_export")
        return pa.RecordBatch._import_from_c(C.addressof(arr), schema)
    sch = _abi.ArrowSchema()
    raise_status(L.murr_arrow_export(outs, k, names, C.byref(arr), C.byref(sch)), what="murr_arrow_export")
    return pa.RecordBatch._import_from_c(C.addressof(arr), C.addressof(sch))


def c_names(names) -> "C.Array":
    """Column names as the const char* const* murr_arrow_export takes."""
    return (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])


def host_array_to_arrow(h) -> pa.Array:
    """murr_host_array_t -> pyarrow Array (copies out of the builder's pinned memory)."""
    n, dt = h.length, DTypeName(h.dtype)
    validity = _copy(h.validity, (n + 7) // 8) if h.validity else None
    if dt == DTypeName.Utf8:
        offs = _copy(h.offsets, (n + 1) * 4)
        data = _copy(h.values, h.values_len)
        return pa.Array.from_buffers(pa.string(), n, [validity, offs, data], null_count=h.null_count)
    vals = _copy(h.values, h.values_len)
    return pa.Array.from_buffers(dt.arrow_dtype(), n, [validity, vals], null_count=h.null_count)


def host_array_buffers(h) -> dict:
    """murr_host_array_t -> raw buffer dict (for bit-exact parity checks)."""
    n = h.length
    out = {"dtype": h.dtype, "length": n, "null_count": h.null_count,
           "validity": C.string_at(h.validity, (n + 7) // 8) if h.validity else None,
           "values": C.string_at(h.values, h.values_len) if h.values_len else b"",
           "offsets": None}
    if h.dtype == int(DTypeName.Utf8):
        out["offsets"] = np.frombuffer(C.string_at(h.offsets, (n + 1) * 4), dtype=np.int32).copy()
    return out


class HostStream:
    """Batch reads back to back, host memory in and out (murr_hstream_*): the
    H2D of batch i+1, the decode of batch i and the D2H of batch i-1 overlap
    on `depth` slots, each with its own stream and reused buffers.

    submit(data, row_off) enqueues one host block (numpy uint8 blob bytes,
    uint64 row offsets; an empty row is a missing key) and returns at once;
    next() waits for the oldest submitted block and returns its decoded arrays
    as murr_host_array_t (valid until `depth` more submits) -- or, with
    arrow=True, as a RecordBatch (copied out).  `pinned=True` tells the
    library the buffers are pinned (HostBuffer / murr_host_alloc): they are
    copied to the device straight from there and must stay unchanged until
    next() returns that block."""

    def __init__(self, segment: SegmentSchema, columns, depth: int = 3, ctx=None):
        self.segment = segment
        self.columns = list(columns)
        self.ctx = ctx or default_context()
        self.L = self.ctx.L
        proj = [c.index if isinstance(c, SegmentColumnSchema) else int(c) for c in self.columns]
        self._proj = (C.c_uint32 * max(len(proj), 1))(*proj)
        self._nproj = len(proj)
        h = C.c_void_p()
        raise_status(self.L.murr_hstream_new(self.ctx.h, C.byref(segment.c), self._proj, self._nproj, int(depth),
                                             C.byref(h)), what="murr_hstream_new")
        self.h = h
        self.depth = depth
        self._keep = {}  # submit sequence -> caller buffers kept alive until returned
        self._seq = self._done = 0
        self._err = _abi.Error()

    def submit(self, data, row_off, pinned: bool = False):
        """One batch: rows back to back at `data`, row_off (n + 1 entries) as
        u64, or as u32 (murr_hstream_submit32: half the offset bytes over
        PCIe) when row_off is a uint32 array."""
        w32 = getattr(row_off, "dtype", None) == np.uint32
        row_off = np.ascontiguousarray(row_off, dtype=np.uint32 if w32 else np.uint64)
        n = row_off.size - 1
        if n < 0:
            raise ValueError("row_off needs n_rows + 1 entries")
        dptr = data.ctypes.data if hasattr(data, "ctypes") else int(data)
        err = _abi.Error()
        fn = self.L.murr_hstream_submit32 if w32 else self.L.murr_hstream_submit
        raise_status(fn(self.h, dptr, row_off.ctypes.data, n, 1 if pinned else 0, C.byref(err)), err,
                     "murr_hstream_submit")
        self._keep[self._seq] = (data, row_off) if pinned else None
        self._seq += 1

    def next(self, arrow: bool = False):
        outs = (_abi.HostArray * self._nproj)()
        st = self.L.murr_hstream_next(self.h, outs, C.byref(self._err))
        self._keep.pop(self._done, None)
        self._done += 1
        raise_status(st, self._err, "murr_hstream_next")
        if not arrow:
            return outs
        if getattr(self, "_arrow_schema", None) is None:
            fields = []
            for col in self.columns:
                seg_col = col if isinstance(col, SegmentColumnSchema) else self.segment.columns[int(col)]
                fields.append(pa.field(seg_col.name, seg_col.dtype.arrow_dtype(), True))
            self._arrow_schema = pa.schema(fields)
            self._cnames = c_names(self._arrow_schema.names)
            rb = host_arrays_to_batch(outs, self._nproj, self._cnames)
            self._batch_schema = rb.schema  # (the later batches import against it)
            return rb
        return host_arrays_to_batch(outs, self._nproj, self._cnames, self._batch_schema)

    @property
    def pending(self) -> int:
        return self._seq - self._done

    def stats(self) -> dict:
        s = _abi.HStreamStats()
        raise_status(self.L.murr_hstream_stats(self.h, C.byref(s)), what="murr_hstream_stats")
        return {f: getattr(s, f) for f, _ in s._fields_}

    def close(self):
        if getattr(self, "h", None):
            self.L.murr_hstream_free(self.h)
            self.h = None
        self._keep.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBuffer:
    """Pinned host memory of the library (murr_host_alloc) as a numpy uint8
    array: the form of a block cache whose blocks the GPU copies directly."""

    def __init__(self, nbytes: int, ctx=None):
        self.ctx = ctx or default_context()
        p = C.c_void_p()
        raise_status(self.ctx.L.murr_host_alloc(self.ctx.h, max(int(nbytes), 1), C.byref(p)), what="murr_host_alloc")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.nbytes, 1)).from_address(self.ptr))[: self.nbytes]

    def close(self):
        if self.ptr and self.ctx.h:
            self.ctx.L.murr_host_free(self.ctx.h, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
