"""One table over several GPUs of one process, read without a collective
(SURVEY.md §8(e) mode 2).

Rows are owned by key: shard_of(key) (fmix64 of FNV-1a, murr_shard_of) picks
the GPU, and each GPU holds its shard as a ResidentTable (blob arena + device
key index).  Table::read (src/io/table/mod.rs:114-129) over the whole table:

1. the caller's keys are routed to their owner shards on the host;
2. every shard looks its keys up and gathers their row blobs on its own GPU
   (murr_index_gather; a miss is an empty row);
3. the gathered blocks are copied to the home GPU, back to back (peer copies
   over xGMI, murr_memcpy_peer -- point to point, no collective);
4. one gather on the home GPU puts the rows in caller order
   (murr_index_gather_copy: row i of the read is the gathered row of key i;
   the positional contract of the reference store,
   src/io/store/rocksdb/mod.rs:368-399);
5. one decode there (murr_decode_blocks) gives the Arrow batch.

Only row blobs cross GPUs, once each, and no GPU waits on another except for
its own peer copy.  Writes route every row to its owner (route_batch), so a
key written again lands on the shard that holds it and the later write wins
(src/io/store/memory.rs:47-60).
"""
from __future__ import annotations

import numpy as np
import pyarrow as pa

from .device import DecodeOutputs, DeviceBlock, decode_blocks, download_array
from .errors import raise_status
from .resident import ResidentTable, _null_dict, host_batch
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
        req = self.shards[0]._resolve(columns)
        nq = len(keys)
        owner = shard_of(keys, self.nshards)
        home = self.home
        L = home.L
        # 2. per shard: gathered block of its keys (caller order within the shard)
        parts = []  # (shard, positions, data buffer, host offsets)
        for s, shard in enumerate(self.shards):
            pos = np.flatnonzero(owner == s)
            if pos.size == 0 or shard.index is None:
                continue
            blk, keep = shard.gather([keys[i] for i in pos])
            offs = blk.row_off.download(8 * (pos.size + 1)).view(np.uint64).copy()
            parts.append((s, pos, blk, offs, keep))
        if not parts:
            return req, [_null_dict(c.dtype, nq) for c in req]
        # 3. peer copies to home, back to back (16-B aligned bases)
        bases, total = [], 0
        for _, pos, _, offs, _ in parts:
            bases.append(total)
            total += (int(offs[-1]) + 15) & ~15
        arena = home.alloc(max(total, 16) + 16)
        for (s, pos, blk, offs, _), base in zip(parts, bases):
            nb = int(offs[-1])
            src_ctx = self.contexts[s]
            raise_status(L.murr_memcpy_peer(home.h, arena.ptr + base, blk.data.ptr, src_ctx.device, nb),
                         what="murr_memcpy_peer")
        # 4. caller-order gather on home: row i = gathered row of key i
        row_start = np.zeros(nq + 1, np.uint64)
        sizes = np.zeros(nq, np.uint64)
        rows = np.zeros(nq, np.uint32)
        cat_off, nrows = [], 0
        for (s, pos, blk, offs, _), base in zip(parts, bases):
            cat_off.append(offs[:-1] + np.uint64(base))
            sizes[pos] = np.diff(offs)
            rows[pos] = np.arange(nrows, nrows + pos.size, dtype=np.uint32)
            nrows += pos.size
        owned = np.zeros(nq, bool)
        for _, pos, _, _, _ in parts:
            owned[pos] = True
        rows[~owned] = 0xFFFFFFFF  # a shard with nothing written yet: the key is missing
        cat = np.concatenate(cat_off + [np.zeros(1, np.uint64)])
        np.cumsum(sizes, out=row_start[1:])
        d_rows, d_cat, d_out_off = home.upload(rows), home.upload(cat), home.upload(row_start)
        nb = int(row_start[-1])
        data = home.alloc(max(nb, 16) + 16)
        if nq:
            raise_status(L.murr_index_gather_copy(home.h, d_rows.ptr, nq, arena.ptr, d_cat.ptr, d_out_off.ptr,
                                                  data.ptr), what="murr_index_gather_copy")
        # 5. one decode on home
        blk = DeviceBlock(data, d_out_off, nq, max(nb, 16))
        proj = [c.index for c in req]
        outs = DecodeOutputs(home, self.segment, proj, [blk])
        decode_blocks(home, self.segment, proj, [blk], outs)
        return req, [download_array(home, outs.array(0, p), int(c.dtype), nq) for p, c in enumerate(req)]
