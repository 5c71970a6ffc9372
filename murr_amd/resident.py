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
appends like MemoryStore::write (src/io/store/memory.rs:47-60): the batch is
encoded on the device straight onto the tail of a blob arena
(murr_encode_batch_at; arena and row offsets grow by doubling) and only its
keys go into the index (murr_index_append: a key written again maps to its
new row, later write wins).  An append costs in proportion to the batch.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pyarrow as pa

from . import _abi
from .device import Context, DecodeOutputs, DecodePlan, DeviceBlock, decode_blocks, download_array
from .errors import SegmentError, raise_status
from .row import c_names, host_arrays_to_arrow, host_arrays_to_batch
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

    def __init__(self, ctx: Context, keys: pa.Array | None = None, *, device_keys=None):
        """Over a host key column, or device_keys = (data DeviceBuffer, int32
        offsets DeviceBuffer, n) already in HBM."""
        self.ctx = ctx
        if device_keys is not None:
            data, offs, self.n = device_keys
        else:
            self.n = len(keys)
            data, offs = _upload_utf8(ctx, keys)
        h = C.c_void_p()
        err = _abi.Error()
        st = ctx.L.murr_index_build(ctx.h, data.ptr, offs.ptr, 0, self.n, C.byref(h), C.byref(err))
        raise_status(st, err, "murr_index_build")
        self.h = h.value
        if device_keys is None:
            data.free()
            offs.free()

    def append(self, keys: pa.Array):
        """murr_index_append: rows n .. n + len(keys) - 1."""
        data, offs = _upload_utf8(self.ctx, keys)
        err = _abi.Error()
        st = self.ctx.L.murr_index_append(self.ctx.h, self.h, data.ptr, offs.ptr, 0, len(keys), C.byref(err))
        raise_status(st, err, "murr_index_append")
        self.n += len(keys)
        data.free()
        offs.free()

    def cache_rows(self, row_off, row_ulen, nutf8: int):
        """murr_index_cache_rows: the rows added since the last call into the
        slot cache (row offsets and sizes, and utf8 string bytes)."""
        err = _abi.Error()
        st = self.ctx.L.murr_index_cache_rows(self.ctx.h, self.h, row_off.ptr,
                                              row_ulen.ptr if row_ulen is not None else None, nutf8, C.byref(err))
        raise_status(st, err, "murr_index_cache_rows")

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


def row_sizes(segment, arrays) -> np.ndarray:
    """Blob bytes of every row of a batch (WriteRow, src/io/row/write.rs:19-52):
    bs + cap, plus 4 + len per non-null utf8 cell.  Host arithmetic on the Arrow
    offsets and validity only."""
    n = len(arrays[0]) if arrays else 0
    size = np.full(n, segment.bitset_size + segment.capacity, np.int64)
    for col, a in zip(segment.columns, arrays):
        if col.dtype != DTypeName.Utf8 or n == 0:
            continue
        offs = np.frombuffer(a.buffers()[1], np.int32)[a.offset:a.offset + n + 1].astype(np.int64)
        lens = np.diff(offs) + 4
        if a.null_count:
            valid = np.unpackbits(np.frombuffer(a.buffers()[0], np.uint8), bitorder="little")[a.offset:a.offset + n]
            lens = lens * valid
        size += lens
    return size


def _key_array(keys) -> pa.Array:
    """Query keys as an Arrow utf8/binary array (the bytes are what is hashed)."""
    try:
        return pa.array(keys, pa.string())
    except (TypeError, pa.ArrowInvalid):
        return pa.array([k.encode() if isinstance(k, str) else bytes(k) for k in keys], pa.binary())


# Gathers whose worst case (keys x longest row) is above this size first look
# the rows up and size the block exactly (one 8-byte read-back), then copy.
TWO_PHASE_BYTES = 64 << 20
# utf8 index stride of the resident arena (murr_utf8_index_update): every
# UIDX_STRIDE rows, each utf8 column's string bytes so far (0.0156 B per row
# and column), so a whole-table scan decodes on the whole GPU in one pass, cut
# into virtual blocks on index strides.  512, as murr_encode_block's default:
# round 4 had moved it to 128 for its dynamic tail (one-tile claims); with the
# static deal the config D shard scans in 0.0748 ms at 512 against 0.0752 at
# 128 (one lane; 0.0566 vs 0.0578 per step with two), interleaved on one box
# (profiles/r05/ab_stride.txt), with a quarter of the index.  A table can
# pick another (uidx_stride).
UIDX_STRIDE = 512
# utf8 columns a prepared read's gather indexes (kGatherMaxU, murr_internal.h)
ROW_ULEN_MAX = 4


def read_capacity(nq: int) -> int:
    """The key-count class of a prepared read: 64, or the next power of two
    (a run of nq keys decodes this many rows; the rest are misses)."""
    return 64 if nq <= 64 else 1 << (int(nq) - 1).bit_length()


class ReadPlan:
    """murr_read_plan_t: Table::read of up to `cap` keys with one projection,
    prepared once over a resident table's current state (include/murr_codec.h).
    run(): host keys -> host arrays (pinned, valid until the next run);
    run_device(): device keys -> device arrays.  One enqueue and one wait per
    run, no descriptor upload and no copy engine."""

    def __init__(self, rt: "ResidentTable", proj, cap: int):
        self.ctx, self.cap, self.nproj = rt.ctx, int(cap), len(proj)
        L = self.ctx.L
        pj = (C.c_uint32 * len(proj))(*proj)
        h = C.c_void_p()
        raise_status(L.murr_read_plan_new(self.ctx.h, C.byref(rt.segment.c), rt.index.h, rt.arena.ptr,
                                          rt.row_off.ptr, rt.ulen.ptr if rt.ulen is not None else None,
                                          rt.used, rt.max_row, pj, len(proj), self.cap,
                                          C.byref(h)), what="murr_read_plan_new")
        self.h = h
        self.host_outs = (_abi.HostArray * len(proj))()
        self.dev_outs = (_abi.Array * len(proj))()
        self.err = _abi.Error()

    def run(self, q: pa.Array):
        """Keys as an Arrow utf8/binary array -> the plan's host arrays."""
        if self.h is None:
            raise SegmentError("read plan closed (the table was written since it was made)")
        kb = q.buffers()
        nq = len(q)
        st = self.ctx.L.murr_read_plan_run(self.h, kb[2].address if nq and kb[2] is not None else None,
                                           kb[1].address if nq else None, q.offset, nq, self.host_outs,
                                           C.byref(self.err))
        raise_status(st, self.err, "murr_read_plan_run")
        return self.host_outs

    def run_device(self, q_data: int, q_offsets: int, nq: int):
        """Keys in device memory (Arrow utf8 layout) -> the plan's device arrays (n = nq)."""
        if self.h is None:
            raise SegmentError("read plan closed (the table was written since it was made)")
        st = self.ctx.L.murr_read_plan_run_device(self.h, q_data, q_offsets, nq, self.dev_outs, C.byref(self.err))
        raise_status(st, self.err, "murr_read_plan_run_device")
        return self.dev_outs

    def close(self):
        if self.h is not None and self.ctx.h:
            self.ctx.L.murr_read_plan_free(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResidentTable:
    """Table (src/io/table/mod.rs:20-155) whose rows stay in HBM."""

    def __init__(self, table: TableSchema, ctx: Context | None = None, name: str = "resident",
                 uidx_stride: int = UIDX_STRIDE):
        self.t = Table(Store(), name, table, ctx)  # schema, validation, column resolution
        self.stride = int(uidx_stride)
        self.ctx = self.t.ctx
        self.segment = self.t.segment
        self.t.prepare()  # kernels compiled at open, never on the read path
        self.index = None
        self.arena = None      # row blobs back to back
        self.arena_cap = 0
        self.used = 0          # arena bytes written
        self.row_off = None    # n + 1 u64 offsets into the arena
        self.off_cap = 0       # entries
        self.n = 0
        self.max_row = 0
        self._reader = None    # murr_reader_t: scratch of the one-call host read
        self._schemas = {}     # read(): per requested column list, its names (C strings) and batch schema
        self.uidx = None       # utf8 index of the arena (every self.stride rows), kept with every write
        self.uidx_cap = 0      # entries
        # per-row utf8 string bytes (murr_utf8_row_lengths, [n][nutf8] u32),
        # kept with every write for layouts of 1 .. ROW_ULEN_MAX utf8 columns:
        # a prepared read's gather indexes its block with them (one-pass decode)
        self.nutf8 = sum(1 for c in self.segment.columns if c.dtype == DTypeName.Utf8)
        self.ulen = None
        self.ulen_cap = 0      # rows
        self._scan_plans = {}  # id(outs) (None: the plan's own outputs) -> (key, DecodePlan) of scan_device
        self._read_plans = {}  # (projection, capacity) -> ReadPlan over the table state _rp_state
        self._rp_state = None

    def __del__(self):
        try:
            for p in self._read_plans.values():
                p.close()
            self._read_plans = {}
            if self._reader is not None and self.ctx.h:
                self.ctx.L.murr_reader_free(self._reader)
                self._reader = None
        except Exception:
            pass

    @property
    def blob(self):
        return self.arena

    def _grow(self, blob_need: int, rows_need: int):
        """Arena and offsets room for blob_need more bytes and rows_need more
        rows (doubling, old contents copied)."""
        need = self.used + blob_need + 16
        if need > self.arena_cap:
            cap = max(need, 2 * self.arena_cap, 1 << 16)
            arena = self.ctx.alloc(cap)
            if self.arena is not None:
                arena.copy_from(self.arena, self.used)
                self.arena.free()
            self.arena, self.arena_cap = arena, cap
        need = self.n + rows_need + 1
        if need > self.off_cap:
            cap = max(need, 2 * self.off_cap, 1024)
            offs = self.ctx.alloc(8 * cap)
            if self.row_off is not None:
                offs.copy_from(self.row_off, 8 * (self.n + 1))
                self.row_off.free()
            self.row_off, self.off_cap = offs, cap

    def write(self, batch: pa.RecordBatch):
        """Table::write into the resident set (validation as table/mod.rs:54-96,
        append as memory.rs:47-60)."""
        keys, arrays = self.t.validate(batch)
        m = batch.num_rows
        if m == 0:
            return
        self._drop_read_plans()  # (before _grow can free the arena they point at)
        sizes = row_sizes(self.segment, arrays)
        bound = int(sizes.sum())
        self._grow(bound, m)
        cols = [_column_dict(self.ctx, a) for a in arrays]
        cin = (_abi.ColIn * max(len(cols), 1))()
        for i, c in enumerate(cols):
            cin[i].values = c["values"].ptr
            cin[i].validity = c["validity"].ptr if c["validity"] is not None else None
            cin[i].offsets = c["offsets"].ptr if c["offsets"] is not None else None
            cin[i].offset = int(c["offset"])
        blen = C.c_uint64()
        err = _abi.Error()
        st = self.ctx.L.murr_encode_batch_at(self.ctx.h, C.byref(self.segment.c), cin, m,
                                             self.arena.ptr + self.used, self.arena_cap - self.used,
                                             self.row_off.ptr + 8 * self.n, self.used, C.byref(blen),
                                             C.byref(err))
        raise_status(st, err, "murr_encode_batch_at")
        assert blen.value == bound, (blen.value, bound)
        if self.index is None:
            self.index = DeviceIndex(self.ctx, keys)
        else:
            self.index.append(keys)
        n_old = self.n
        self.used += blen.value
        self.n += m
        self.max_row = max(self.max_row, int(sizes.max()))
        self._index_tail(n_old)

    def _index_tail(self, n_old: int):
        """Extend the arena's utf8 index over rows n_old .. n (the written
        block's index, kept as the table grows: only the new rows are read),
        and the per-row utf8 string bytes over the same rows."""
        L, seg = self.ctx.L, self.segment
        if 1 <= self.nutf8 <= ROW_ULEN_MAX:
            if self.n > self.ulen_cap:
                cap = max(self.n, 2 * self.ulen_cap, 1024)
                buf = self.ctx.alloc(4 * self.nutf8 * cap)
                if self.ulen is not None and n_old:
                    buf.copy_from(self.ulen, 4 * self.nutf8 * n_old)
                    self.ulen.free()
                self.ulen, self.ulen_cap = buf, cap
            blk = _abi.Block(self.arena.ptr, self.row_off.ptr, self.n, self.used)
            raise_status(L.murr_utf8_row_lengths(self.ctx.h, C.byref(seg.c), C.byref(blk), n_old, self.ulen.ptr),
                         what="murr_utf8_row_lengths")
        # the index's slot cache: each slot's row offset, size (and string bytes)
        self.index.cache_rows(self.row_off, self.ulen, self.nutf8 if self.ulen is not None else 0)
        need = int(L.murr_utf8_index_len(C.byref(seg.c), self.n, self.stride))
        if need == 0:
            return
        if need > self.uidx_cap:
            cap = max(need, 2 * self.uidx_cap, 64)
            buf = self.ctx.alloc(8 * cap)
            if self.uidx is not None and n_old:
                buf.copy_from(self.uidx, 8 * int(L.murr_utf8_index_len(C.byref(seg.c), n_old, self.stride)))
                self.uidx.free()
            self.uidx, self.uidx_cap = buf, cap
        blk = _abi.Block(self.arena.ptr, self.row_off.ptr, self.n, self.used)
        raise_status(L.murr_utf8_index_update(self.ctx.h, C.byref(seg.c), C.byref(blk), n_old, self.stride,
                                              self.uidx.ptr), what="murr_utf8_index_update")

    def load_sst(self, entries):
        """Rehydrate an empty table from SST entries decoded on the device
        (murr_amd.sst.decode): the values are the table's row blobs and become
        the arena as they lie, the user keys go into the device index.  The
        entries must be live rows (value type kTypeValue, as in a compacted
        bottommost file).  A key seen more than once maps to its entry with
        the highest sequence number (RocksDB keeps a key's versions newest
        first within a file, and overlapping files repeat keys in any order;
        murr_index_prefer_seq).  Nothing but the value lengths and types
        crosses to the host."""
        if self.n:
            raise SegmentError("load_sst rehydrates an empty resident table")
        self._drop_read_plans()
        n = entries.n
        if n == 0:
            return
        types = entries.types.download(n)
        if (types != 1).any():
            i = int(np.flatnonzero(types != 1)[0])
            raise SegmentError(f"entry {i} has value type {int(types[i])}: only live values (type 1) rehydrate")
        lens = np.diff(entries.value_offsets.download(8 * (n + 1)).view(np.uint64))
        self.index = DeviceIndex(self.ctx, device_keys=(entries.keys, entries.key_offsets, n))
        err = _abi.Error()
        raise_status(self.ctx.L.murr_index_prefer_seq(self.ctx.h, self.index.h, entries.seqs.ptr, C.byref(err)),
                     err, "murr_index_prefer_seq")
        self.arena, self.arena_cap = entries.values, entries.value_bytes + 16
        self.row_off, self.off_cap = entries.value_offsets, n + 1
        self.used, self.n = entries.value_bytes, n
        self.max_row = int(lens.max())
        self._index_tail(0)

    def gather(self, keys):
        """Lookup + gather on the device: a DeviceBlock of the rows of `keys` in
        caller order (a miss = an empty row).  The block is sized from keys x
        the longest row when that is small, else exactly (two phases)."""
        if self.index is None:
            raise SegmentError("resident table is empty")
        nq = len(keys)
        if isinstance(keys, pa.Array):  # (an Arrow key array as it is: its bytes are what is hashed)
            q = keys.view(pa.binary()) if pa.types.is_string(keys.type) else keys
        else:
            q = pa.array([k.encode() if isinstance(k, str) else bytes(k) for k in keys], pa.binary())
        qd, qo = _upload_utf8(self.ctx, q.view(pa.string()))
        offs = self.ctx.alloc((nq + 1) * 8)
        needed = self.ctx.alloc(8)
        bound = max(nq * self.max_row, 16)
        L = self.ctx.L
        if bound <= TWO_PHASE_BYTES:
            data = self.ctx.alloc(bound + 16)
            st = L.murr_index_gather(self.ctx.h, self.index.h, qd.ptr, qo.ptr, nq, self.arena.ptr, self.row_off.ptr,
                                     data.ptr, bound, offs.ptr, None, needed.ptr)
            raise_status(st, what="murr_index_gather")
            # the decode's tile sizing hint: the mean row (data_bytes is never read past)
            hint = min(bound, max(16, int(self.used / max(self.n, 1) * nq)))
            return DeviceBlock(data, offs, nq, hint), (qd, qo)
        rows = self.ctx.alloc(max(nq, 1) * 4)
        st = L.murr_index_gather(self.ctx.h, self.index.h, qd.ptr, qo.ptr, nq, self.arena.ptr, self.row_off.ptr,
                                 None, 0, offs.ptr, rows.ptr, needed.ptr)
        raise_status(st, what="murr_index_gather")
        nb = int(needed.download(8).view(np.uint64)[0])
        data = self.ctx.alloc(max(nb, 16) + 16)
        st = L.murr_index_gather_copy(self.ctx.h, rows.ptr, nq, self.arena.ptr, self.row_off.ptr, offs.ptr, data.ptr)
        raise_status(st, what="murr_index_gather_copy")
        return DeviceBlock(data, offs, nq, max(nb, 16)), (qd, qo, rows)

    def block(self) -> DeviceBlock:
        """The whole arena as one decode block, with its utf8 index."""
        return DeviceBlock(self.arena, self.row_off, self.n, self.used, self.uidx,
                           self.stride if self.uidx is not None else 0)

    def scan_device(self, columns, outs: DecodeOutputs | None = None) -> DecodeOutputs:
        """Every row of the table, decoded on the device in one launch over the
        whole arena (cut on its utf8 index, so every CU takes part): Arrow
        buffers in HBM.  `outs` (from an earlier scan of the same columns and
        row count) is reused.  The bulk read of SURVEY.md §8(e) mode 1: a GPU
        decodes its whole shard."""
        return self.scan_device_async(columns, outs).wait()

    def scan_device_async(self, columns, outs: DecodeOutputs | None = None, ctx: Context | None = None) -> DecodePlan:
        """scan_device's launch only (murr_decode_run_async): returns the
        prepared plan, whose wait() finishes the scan and returns its outputs.
        A caller alternating two `outs` launches the next scan before waiting
        for the previous one; each `outs` keeps its own prepared plan.
        `ctx`: another context on the table's device (its own stream) to
        launch on, so back-to-back scans on two contexts overlap -- the next
        scan's workgroups start on the CUs the previous one's tail leaves idle
        (bench.py --config D --lanes 2).  The arena is only read."""
        if self.n == 0:
            self._resolve(columns)  # (an unknown column is reported first)
            raise SegmentError("resident table is empty")
        # the plan's key: columns, table state, the context's options (a
        # repeated scan costs a tuple compare here and one library call)
        lane = ctx or self.ctx
        if lane.device != self.ctx.device:
            raise ValueError("scan_device_async: the context must be on the table's device")
        state = (tuple(columns), self.arena.ptr, self.row_off.ptr, self.uidx.ptr if self.uidx is not None else 0,
                 self.n, self.used, getattr(lane, "opts_gen", 0), id(lane))
        slot = id(outs) if outs is not None else None
        plan = self._scan_plans.get(slot)
        if plan is None or plan[0] != state or (outs is not None and outs is not plan[1].outs):
            proj = [c.index for c in self._resolve(columns)]
            # prepared once per (columns, table state, outputs): a repeated
            # scan is one launch and one small read-back (murr_decode_run).
            # Without `outs` the plan's own outputs are reused (valid until
            # the next scan).
            if plan is not None:
                plan[1].close()
            if len(self._scan_plans) >= 4:  # a few output sets at most: evict
                # one, preferring a plan with no run in flight (closing an
                # in-flight plan finishes its run first; its wait() still
                # returns that run's outputs)
                cand = [k for k in self._scan_plans if k != slot]
                idle = [k for k in cand if not self._scan_plans[k][1].inflight]
                if cand:
                    self._scan_plans.pop((idle or cand)[0])[1].close()
            blk = self.block()
            p = DecodePlan(lane, self.segment, proj, [blk], outs or DecodeOutputs(lane, self.segment, proj, [blk]))
            self._scan_plans[slot] = plan = (state, p)
        plan[1].run_async()
        return plan[1]

    def scan(self, columns) -> pa.RecordBatch:
        """scan_device, brought to the host as a RecordBatch (rows in write
        order; a key written twice appears twice, as in the arena)."""
        req = self._resolve(columns)
        if self.n == 0:
            return host_batch(req, [_null_dict(c.dtype, 0) for c in req])
        outs = self.scan_device(columns)
        return host_batch(req, [download_array(self.ctx, outs.array(0, p), int(c.dtype), self.n)
                                for p, c in enumerate(req)])

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
        if self.index is None or nq == 0:
            return req, [_null_dict(c.dtype, nq) for c in req]
        blk, _keep = self.gather(keys)
        proj = [c.index for c in req]
        outs = DecodeOutputs(self.ctx, self.segment, proj, [blk])
        decode_blocks(self.ctx, self.segment, proj, [blk], outs)
        return req, [download_array(self.ctx, outs.array(0, p), int(c.dtype), nq) for p, c in enumerate(req)]

    def _drop_read_plans(self):
        """A write changes the arena, offsets and index the prepared reads
        point at (and may free them): every plan is closed now, so a caller
        still holding one gets an error from its run, not stale memory."""
        for p in self._read_plans.values():
            p.close()
        self._read_plans = {}
        self._rp_state = None

    def read_plan(self, columns, nq: int) -> ReadPlan | None:
        """The prepared read (ReadPlan) for these columns and nq keys over the
        table as it is now: made at the first read of its key-count class
        (read_capacity) and reused until a write changes the table.  None
        when nq x the longest row passes TWO_PHASE_BYTES (such reads size
        their gather exactly, murr_reader_read)."""
        if self.index is None or nq == 0:
            return None
        proj = tuple(c.index for c in self._resolve(columns))
        cap = read_capacity(nq)
        if cap * max(self.max_row, 1) > TWO_PHASE_BYTES:
            return None
        state = (self.arena.ptr, self.row_off.ptr, self.ulen.ptr if self.ulen is not None else 0, self.n, self.used,
                 self.max_row)
        if state != self._rp_state:  # the table changed since the plans were made: every plan is stale
            self._drop_read_plans()
            self._rp_state = state
        plan = self._read_plans.pop((proj, cap), None)
        if plan is None:
            if len(self._read_plans) >= 8:  # least recently used first
                self._read_plans.pop(next(iter(self._read_plans))).close()
            plan = ReadPlan(self, list(proj), cap)
        self._read_plans[(proj, cap)] = plan  # (most recently used last)
        return plan

    def read(self, keys, columns) -> pa.RecordBatch:
        """Table::read (table/mod.rs:114-129) with the store lookup on the
        device: a prepared read (ReadPlan: lookup + gather + decode + the
        arrays to pinned memory, one enqueue and one wait), or for a read too
        large for one (murr_reader_read) the one-call read with exact sizing."""
        req = self._resolve(columns)
        nq = len(keys)
        if self.index is None:
            return host_batch(req, [_null_dict(c.dtype, nq) for c in req])
        L = self.ctx.L
        q = keys if isinstance(keys, pa.Array) else _key_array(keys)
        plan = self.read_plan(columns, nq)
        if plan is not None:
            outs = plan.run(q)
        else:
            if self._reader is None:
                h = C.c_void_p()
                raise_status(L.murr_reader_new(self.ctx.h, C.byref(self.segment.c), C.byref(h)),
                             what="murr_reader_new")
                self._reader = h
            kb = q.buffers()
            proj = (C.c_uint32 * len(req))(*[c.index for c in req])
            outs = (_abi.HostArray * len(req))()
            err = _abi.Error()
            st = L.murr_reader_read(self._reader, self.index.h, self.arena.ptr, self.row_off.ptr, self.used,
                                    self.max_row, kb[2].address if nq and kb[2] is not None else None,
                                    kb[1].address if nq else None, q.offset, nq, proj, len(req), outs, C.byref(err))
            raise_status(st, err, "murr_reader_read")
        # the RecordBatch through the Arrow C Data Interface: the library
        # copies the arrays out of its pinned memory into an export pyarrow
        # imports in one call (one Array.from_buffers per column cost ~4x more)
        key = tuple(c.name for c in req)
        ent = self._schemas.get(key)
        if ent is None:  # (the field names as C strings, and the first batch's schema, once per column list)
            names = c_names(list(key))
            rb = host_arrays_to_batch(outs, len(req), names)
            self._schemas[key] = (names, rb.schema)
            return rb
        return host_arrays_to_batch(outs, len(req), ent[0], ent[1])

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
        blk, _keep = self.gather(keys)
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
