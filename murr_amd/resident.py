"""A table held in HBM: row blobs + a device key index.

`ResidentTable.read` runs the whole Table::read on the device: the query keys
go through the index (murr_index_gather: hash lookup, then the hit rows
gathered back to back in caller order, a miss as an empty row) and the block
into the decode kernel, so there is no host round trip between the lookup and
the Arrow output.  It is the device-resident counterpart of Table::read over
RocksDBStore / MemoryStore (src/io/table/mod.rs:114-129,
src/io/store/rocksdb/mod.rs:241-267, src/io/store/memory.rs:28-45) and answers
exactly as they do: request order, duplicates allowed, missing keys as all-null
rows, later writes of a key win.

`write` keeps Table::write's validation (src/io/table/mod.rs:54-96) and
encodes on the device (murr_encode_batch).  A write appends to the resident
set: the batches are re-encoded together and the index rebuilt, which suits a
bulk-loaded hot set (one load, many reads) rather than a write-heavy table.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pyarrow as pa

from . import _abi
from .device import Context, DecodeOutputs, DeviceBlock, decode_blocks, download_array, encode_batch
from .errors import SegmentError, raise_status
from .schema import DTypeName, TableSchema
from .store import Store
from .table import Table

ROW_MISSING = 0xFFFFFFFF


def _upload_utf8(ctx: Context, arr: pa.Array):
    """A utf8 Arrow array's (data, offsets) as device buffers (offsets from
    element 0, the array offset applied)."""
    arr = arr.cast(pa.string()) if arr.type != pa.string() else arr
    n = len(arr)
    bufs = arr.buffers()
    if bufs[1] is None:
        return ctx.upload(np.zeros(16, np.uint8)), ctx.upload(np.zeros(1, np.int32))
    offs = np.frombuffer(bufs[1], dtype=np.int32)[arr.offset:arr.offset + n + 1]
    base = int(offs[0]) if n else 0
    offs = (offs - base).astype(np.int32)
    data = np.frombuffer(bufs[2], dtype=np.uint8)[base:base + int(offs[-1])] if (n and bufs[2] is not None) \
        else np.zeros(0, np.uint8)
    return ctx.upload(np.concatenate([data, np.zeros(16, np.uint8)])), ctx.upload(offs)


def _column_dict(ctx: Context, arr: pa.Array) -> dict:
    """One Arrow input column as device buffers for device.encode_batch."""
    bufs = arr.buffers()
    d = {"offset": arr.offset, "validity": None, "offsets": None, "utf8_bytes": 0}
    if bufs[0] is not None and arr.null_count:
        d["validity"] = ctx.upload(np.frombuffer(bufs[0], dtype=np.uint8))
    if arr.type == pa.string():
        offs = np.frombuffer(bufs[1], dtype=np.int32)
        d["offsets"] = ctx.upload(offs)
        data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
        d["values"] = ctx.upload(np.concatenate([data, np.zeros(16, np.uint8)]))
        d["utf8_bytes"] = int(offs[arr.offset + len(arr)]) if len(arr) else 0
    else:
        d["values"] = ctx.upload(np.concatenate([np.frombuffer(bufs[1], dtype=np.uint8),
                                                 np.zeros(16, np.uint8)]))
    return d


class DeviceIndex:
    """murr_index_t: hash index over a device utf8 key column."""

    def __init__(self, ctx: Context, keys: pa.Array):
        self.ctx = ctx
        self.n = len(keys)
        data, offs = _upload_utf8(ctx, keys)
        h = C.c_void_p()
        err = _abi.Error()
        st = ctx.L.murr_index_build(ctx.h, data.ptr, offs.ptr, 0, self.n, C.byref(h), C.byref(err))
        raise_status(st, err, "murr_index_build")
        self.h = h.value
        data.free()
        offs.free()

    def info(self):
        n, slots = C.c_uint64(), C.c_uint64()
        raise_status(self.ctx.L.murr_index_info(self.h, C.byref(n), C.byref(slots)), what="murr_index_info")
        return n.value, slots.value

    def lookup(self, keys) -> np.ndarray:
        """Rows of `keys` (ROW_MISSING for a miss)."""
        q = pa.array([bytes(k) if not isinstance(k, str) else k.encode() for k in keys], pa.binary())
        qd, qo = _upload_utf8(self.ctx, q.view(pa.string()))
        rows = self.ctx.alloc(max(len(keys), 1) * 4)
        raise_status(self.ctx.L.murr_index_lookup(self.ctx.h, self.h, qd.ptr, qo.ptr, len(keys), rows.ptr),
                     what="murr_index_lookup")
        return rows.download(len(keys) * 4).view(np.uint32)

    def close(self):
        if getattr(self, "h", None):
            self.ctx.L.murr_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResidentTable:
    """Table (src/io/table/mod.rs:20-155) whose rows stay in HBM."""

    def __init__(self, table: TableSchema, ctx: Context | None = None, name: str = "resident"):
        self.t = Table(Store(), name, table, ctx)  # schema, validation, column resolution
        self.ctx = self.t.ctx
        self.segment = self.t.segment
        self.batches = []
        self.index = None
        self.blob = self.row_off = None
        self.n = 0
        self.max_row = 0

    def write(self, batch: pa.RecordBatch):
        """Table::write into the resident set (validation as table/mod.rs:54-96)."""
        self.t.validate(batch)
        batches = self.batches + [batch]
        whole = pa.Table.from_batches(batches).combine_chunks()
        merged = whole.to_batches()[0] if whole.num_rows else batch
        keys, arrays = self.t.validate(merged)
        n = merged.num_rows
        cols = [_column_dict(self.ctx, a) for a in arrays]
        blob, row_off, _ = encode_batch(self.ctx, self.segment, cols, n)
        index = DeviceIndex(self.ctx, keys)
        offs = row_off.download((n + 1) * 8).view(np.uint64)
        self.batches = batches
        self.blob, self.row_off, self.index, self.n = blob, row_off, index, n
        self.max_row = int(np.diff(offs).max()) if n else 0

    def gather(self, keys):
        """Lookup + gather on the device: a DeviceBlock of the rows of `keys` in
        caller order (a miss = an empty row)."""
        nq = len(keys)
        q = pa.array([k.encode() if isinstance(k, str) else bytes(k) for k in keys], pa.binary())
        qd, qo = _upload_utf8(self.ctx, q.view(pa.string()))
        cap = max(nq * self.max_row, 16)
        data = self.ctx.alloc(cap + 16)
        offs = self.ctx.alloc((nq + 1) * 8)
        needed = self.ctx.alloc(8)
        blob = self.blob.ptr if self.blob is not None else None
        row_off = self.row_off.ptr if self.row_off is not None else None
        if self.index is None:
            raise SegmentError("resident table is empty")
        st = self.ctx.L.murr_index_gather(self.ctx.h, self.index.h, qd.ptr, qo.ptr, nq, blob, row_off,
                                          data.ptr, cap, offs.ptr, None, needed.ptr)
        raise_status(st, what="murr_index_gather")
        return DeviceBlock(data, offs, nq, 0), needed, (qd, qo)

    def _resolve(self, columns):
        req = []
        for name in columns:
            idx = self.t.columns.get(name)
            if idx is None:
                raise SegmentError(f"column '{name}' not found")
            req.append(self.segment.columns[idx])
        if not req:
            from .errors import ArrowError
            raise ArrowError("Arrow error: must either specify a row count or at least one column")
        return req

    def read_host(self, keys, columns):
        """Lookup + gather + decode on the device, then D2H: (requested
        SegmentColumnSchema list, host buffer dicts as download_array returns
        them).  A miss is an all-null row (add_empty)."""
        req = self._resolve(columns)
        nq = len(keys)
        if self.index is None:
            return req, [_null_dict(c.dtype, nq) for c in req]
        blk, needed, _keep = self.gather(keys)
        blk.data_bytes = max(nq * self.max_row, 16)
        proj = [c.index for c in req]
        outs = DecodeOutputs(self.ctx, self.segment, proj, [blk])
        decode_blocks(self.ctx, self.segment, proj, [blk], outs)
        assert int(needed.download(8).view(np.uint64)[0]) <= max(nq * self.max_row, 16)
        return req, [download_array(self.ctx, outs.array(0, p), int(c.dtype), nq) for p, c in enumerate(req)]

    def read(self, keys, columns) -> pa.RecordBatch:
        """Table::read (table/mod.rs:114-129) with the store lookup on the device."""
        req, hs = self.read_host(keys, columns)
        return host_batch(req, hs)

    def read_ipc(self, keys, columns, alignment: int = 64) -> bytes:
        """read() as the Arrow IPC stream of the HTTP fetch handler's StreamWriter
        (src/api/http/handlers.rs:88-101), built on the device: lookup + gather +
        decode, then one kernel packs the record-batch message in HBM
        (murr_ipc_batch_device) and one D2H copy brings it back."""
        from . import ipc
        req = []
        for name in columns:
            idx = self.t.columns.get(name)
            if idx is None:
                raise SegmentError(f"column '{name}' not found")
            req.append(self.segment.columns[idx])
        if not req:
            from .errors import ArrowError
            raise ArrowError("Arrow error: must either specify a row count or at least one column")
        nq = len(keys)
        schema = ipc.schema_message(self.segment, req, alignment)
        if self.index is None:
            return ipc.stream(schema, _all_null_message(self.segment, req, nq, alignment))
        blk, needed, _keep = self.gather(keys)
        blk.data_bytes = max(nq * self.max_row, 16)
        proj = [c.index for c in req]
        outs = DecodeOutputs(self.ctx, self.segment, proj, [blk])
        decode_blocks(self.ctx, self.segment, proj, [blk], outs)
        dev, n = ipc.batch_message_device(self.ctx, self.segment, proj, outs, 0, nq, alignment)
        return ipc.stream(schema, ipc.download_message(self.ctx, dev, n))


def _all_null_message(segment, req, n: int, alignment: int) -> bytes:
    """Every key missing (add_empty for each, rocksdb/mod.rs:262-263)."""
    from . import ipc
    nb = (n + 7) // 8
    keep = []
    arr = (_abi.HostArray * len(req))()

    def zeros(k):
        b = C.create_string_buffer(max(k, 1))
        keep.append(b)
        return C.addressof(b)
    for p, c in enumerate(req):
        h = arr[p]
        h.length, h.null_count, h.dtype = n, n, int(c.dtype)
        h.validity = zeros(nb) if n else None
        if c.dtype == DTypeName.Utf8:
            h.offsets, h.values, h.values_len = zeros(4 * (n + 1)), zeros(0), 0
        elif c.dtype == DTypeName.Bool:
            h.values, h.values_len = zeros(nb), nb
        else:
            h.values, h.values_len = zeros(n * c.dtype.size()), n * c.dtype.size()
    return ipc.batch_message_host(segment, req, arr, n, alignment)


def _null_dict(dt: DTypeName, n: int) -> dict:
    nb = (n + 7) // 8
    h = {"dtype": int(dt), "length": n, "null_count": n, "validity": bytes(nb), "offsets": None}
    if dt == DTypeName.Utf8:
        h["offsets"], h["values"] = np.zeros(n + 1, np.int32), b""
    elif dt == DTypeName.Bool:
        h["values"] = bytes(nb)
    else:
        h["values"] = bytes(n * dt.size())
    return h


def host_batch(req, hs) -> pa.RecordBatch:
    """Host buffer dicts -> RecordBatch (nullable fields, no metadata, read.rs:105)."""
    arrays = [_to_arrow(h, c.dtype) for c, h in zip(req, hs)]
    fields = [pa.field(c.name, c.dtype.arrow_dtype(), True) for c in req]
    return pa.RecordBatch.from_arrays(arrays, schema=pa.schema(fields))


def _to_arrow(h: dict, dt: DTypeName) -> pa.Array:
    n = h["length"]
    nb = (n + 7) // 8  # bitmaps come back padded (murr_bitmap_bytes); Arrow's are ceil(n/8)
    validity = pa.py_buffer(h["validity"][:nb]) if h["null_count"] else None
    if dt == DTypeName.Bool:
        return pa.Array.from_buffers(pa.bool_(), n, [validity, pa.py_buffer(h["values"][:nb])],
                                     null_count=h["null_count"])
    if dt == DTypeName.Utf8:
        return pa.Array.from_buffers(pa.string(), n, [validity, pa.py_buffer(h["offsets"].tobytes()),
                                                      pa.py_buffer(h["values"])], null_count=h["null_count"])
    return pa.Array.from_buffers(dt.arrow_dtype(), n, [validity, pa.py_buffer(h["values"])],
                                 null_count=h["null_count"])
