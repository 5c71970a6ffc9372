"""One table over several GPUs of one process, read without a collective
(SURVEY.md §8(e) mode 2).

Rows are owned by key: shard_of(key) (fmix64 of FNV-1a, murr_shard_of) picks
the GPU, and each GPU holds its shard as a ResidentTable (blob arena + device
key index).  Table::read (src/io/table/mod.rs:114-129) over the whole table:

1. the caller's keys are routed to their owner shards on the host and
   uploaded to the home GPU once, grouped by owner;
2. every shard looks its keys up on its own GPU and stream, all at once
   (reading the keys from home memory and writing their rows there, peer
   access over xGMI);
3. the home stream waits on those lookups (events, not the host) and builds
   the caller-order block: each key's row blob is copied straight from its
   shard's arena (murr_multi_gather: row i of the read is the row of key i, a
   miss an empty row -- the positional contract of the reference store,
   src/io/store/rocksdb/mod.rs:368-399);
4. one decode there (murr_decode_blocks) gives the Arrow batch; its wait is
   the read's one host synchronisation.

Only row blobs cross GPUs, once each, no collective runs, and no host round
trip sits between the shards' lookups and the decode.  Writes route every row to its owner (route_batch), so a
key written again lands on the shard that holds it and the later write wins
(src/io/store/memory.rs:47-60).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pyarrow as pa

from . import _abi
from .device import DecodeOutputs, DeviceBlock, decode_blocks, download_array
from .errors import raise_status
from .resident import TWO_PHASE_BYTES, ResidentTable, _null_dict, host_batch
from .schema import TableSchema
from .shard import route_batch, shard_of


class MultiDeviceTable:
    """A table sharded by key over `contexts` (one murr context per GPU; the
    first is home, where reads are assembled and decoded)."""

    def __init__(self, table: TableSchema, contexts, name: str = "multi"):
        if not contexts:
            raise ValueError("no contexts")
        self.contexts = list(contexts)
        self.shards = [ResidentTable(table, ctx, f"{name}.{i}") for i, ctx in enumerate(self.contexts)]
        self.home = self.contexts[0]
        self.segment = self.shards[0].segment
        self.table = table

    @property
    def nshards(self) -> int:
        return len(self.shards)

    def write(self, batch: pa.RecordBatch):
        """Table::write: validation once, then each shard appends its rows."""
        self.shards[0].t.validate(batch)
        for shard, part in zip(self.shards, route_batch(batch, self.table.key, self.nshards)):
            if part.num_rows:
                shard.write(part)

    def read(self, keys, columns) -> pa.RecordBatch:
        req, hs = self.read_host(keys, columns)
        return host_batch(req, hs)

    def read_host(self, keys, columns):
        """The read's columns as host arrays (murr_multi_gather + one decode on
        home).  The host routes the keys and uploads them once, grouped by
        owner; everything after is enqueued on the GPUs' streams with
        stream-to-stream waits, and the host waits once, for the decode."""
        req = self.shards[0]._resolve(columns)
        nq = len(keys)
        home = self.home
        L = home.L
        if nq == 0 or all(sh.index is None for sh in self.shards):
            return req, [_null_dict(c.dtype, nq) for c in req]
        # 1. route: grouped position of every caller query, shard ranges
        kb = pa.array([k.encode() if isinstance(k, str) else bytes(k) for k in keys], pa.binary())
        owner = shard_of(kb, self.nshards)
        order = np.argsort(owner, kind="stable")
        src = np.empty(nq, np.uint32)
        src[order] = np.arange(nq, dtype=np.uint32)
        q_end = np.cumsum(np.bincount(owner, minlength=self.nshards)).astype(np.uint64)
        grouped = kb.take(pa.array(order))
        goff = np.frombuffer(grouped.buffers()[1], np.int32)[grouped.offset: grouped.offset + nq + 1]
        gdat = grouped.buffers()[2]
        gdat = np.frombuffer(gdat, np.uint8) if gdat is not None else np.zeros(0, np.uint8)
        # one upload: [offsets (nq + 1) i32 | src (nq) u32 | key bytes]
        o_src = (4 * (nq + 1) + 15) & ~15
        o_dat = (o_src + 4 * nq + 15) & ~15
        kbytes = gdat[int(goff[0]): int(goff[-1])]
        packed = np.zeros(o_dat + kbytes.size + 16, np.uint8)
        packed[: 4 * (nq + 1)] = (goff - goff[0]).astype(np.int32).view(np.uint8)
        packed[o_src: o_src + 4 * nq] = src.view(np.uint8)
        packed[o_dat: o_dat + kbytes.size] = kbytes
        qbuf = home.upload(packed)
        # 2. lookups on every shard's stream, caller-order block on home
        tab = (_abi.ShardRead * self.nshards)()
        for s_, sh in enumerate(self.shards):
            tab[s_].ctx = self.contexts[s_].h
            tab[s_].index = sh.index.h if sh.index is not None else None
            tab[s_].arena = sh.arena.ptr if sh.index is not None else None
            tab[s_].row_off = sh.row_off.ptr if sh.index is not None else None
            tab[s_].q_end = int(q_end[s_])
        rows = home.alloc(4 * nq)
        out_off = home.alloc(8 * (nq + 1))
        needed = home.alloc(8)
        bound = max(16, nq * max(sh.max_row for sh in self.shards if sh.index is not None))
        two_phase = bound > TWO_PHASE_BYTES
        data = None if two_phase else home.alloc(bound + 16)
        err = _abi.Error()
        raise_status(L.murr_multi_gather(home.h, tab, self.nshards, qbuf.ptr + o_dat, qbuf.ptr, qbuf.ptr + o_src, nq,
                                         rows.ptr, out_off.ptr, data.ptr if data else None, bound, needed.ptr,
                                         C.byref(err)), err, "murr_multi_gather")
        if two_phase:  # the block's size first (one more wait), then its copy
            nb = int(needed.download(8).view(np.uint64)[0])
            data = home.alloc(max(nb, 16) + 16)
            raise_status(L.murr_multi_gather_copy(home.h, tab, self.nshards, qbuf.ptr + o_src, nq, rows.ptr,
                                                  out_off.ptr, data.ptr, C.byref(err)), err, "murr_multi_gather_copy")
            bound = max(nb, 16)
        # 3. one decode on home (its wait is the read's host synchronisation)
        # data_bytes sizes every utf8 values buffer of the decode: a safe upper
        # bound of the gathered bytes (nq x the longest row, at most
        # TWO_PHASE_BYTES here; the exact size on the two-phase path), never a
        # mean-row estimate a read of long rows could outgrow
        blk = DeviceBlock(data, out_off, nq, bound)
        proj = [c.index for c in req]
        outs = DecodeOutputs(home, self.segment, proj, [blk])
        decode_blocks(home, self.segment, proj, [blk], outs)
        self._keep = (qbuf, rows, needed)
        return req, [download_array(home, outs.array(0, p), int(c.dtype), nq) for p, c in enumerate(req)]
