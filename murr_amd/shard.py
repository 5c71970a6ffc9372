"""Sharding across GPUs.

Bulk decode (mode 1, bench.py): one process per GPU, each decoding its own
contiguous key range; no data-path collective.  torch.distributed (gloo, CPU
tensors) carries only the start/stop barriers and the max-over-ranks time /
sum-over-ranks bytes the bench reports: every output cell depends on exactly
one input row (src/io/row/read.rs:85-91) and the utf8 offset prefix is local
to a block.

Random-key reads (mode 2) across one process per GPU (`merge_reads`,
`ShardedResidentTable`): every rank reads the caller's keys against its own
shard and the caller-order batch is the byte-wise sum of the ranks' buffers,
three all-reduces per read (validity / fixed values / bool bitmaps, utf8
lengths, utf8 bytes).  That sum is only correct when every key lives on
exactly one rank, so writes are routed by key (`shard_of`) and `write_shard`
refuses keys this rank does not own.  The collective-free form of mode 2 (one
process driving every GPU: keys routed on the host, rows gathered on their
shard's GPU, one peer-copy gather to the caller's GPU) is
`murr_amd.multigpu.MultiDeviceTable`.
"""
from __future__ import annotations

import os

import numpy as np


def shard_of(keys, nshards: int) -> np.ndarray:
    """Owner shard of every key (murr_shard_of: fmix64 of FNV-1a 64 over the
    key bytes, mod nshards).  `keys`: a pyarrow string/binary array or a list
    of str/bytes."""
    import ctypes as C
    import pyarrow as pa
    from . import _abi
    from .errors import raise_status
    arr = keys if isinstance(keys, pa.Array) else pa.array(
        [k.encode() if isinstance(k, str) else bytes(k) for k in keys], pa.binary())
    if pa.types.is_string(arr.type):
        arr = arr.view(pa.binary())
    n = len(arr)
    out = np.zeros(n, np.uint32)
    if n == 0:
        return out
    bufs = arr.buffers()
    offs = np.frombuffer(bufs[1], np.int32)
    data = np.frombuffer(bufs[2], np.uint8) if bufs[2] is not None else np.zeros(1, np.uint8)
    st = _abi.lib().murr_shard_of(data.ctypes.data, offs.ctypes.data, arr.offset, n, nshards, out.ctypes.data)
    raise_status(st, what="murr_shard_of")
    return out


def check_owned(keys, rank: int, world: int):
    """Raise ValueError unless every key's owner shard is `rank`."""
    owner = shard_of(keys, world)
    bad = np.flatnonzero(owner != rank)
    if bad.size:
        raise ValueError(f"{bad.size} keys belong to other shards (first: row {int(bad[0])} -> shard "
                         f"{int(owner[bad[0]])}); route writes with route_batch")


def route_batch(batch, key: str, nshards: int):
    """Split a RecordBatch by the owner shard of its key column: one batch per
    shard (rows keep their order)."""
    import pyarrow as pa
    owner = shard_of(batch.column(batch.schema.get_field_index(key)), nshards)
    return [batch.take(pa.array(np.flatnonzero(owner == s))) for s in range(nshards)]


def shard_rows(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous key range [start, start + count) of `rank` out of `world`
    over `total` rows (earlier ranks take the remainder, one row each)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


class Group:
    """The bench's process group: None-safe wrappers (world size 1 = no group)."""

    def __init__(self, backend: str = "gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.dist = None
        self.rank, self.local_rank = 0, 0
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group(backend)
            self.dist = dist
            self.rank = dist.get_rank()
            self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM if self.dist else None)

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


# ---- random-key batch read across key-range shards (SURVEY.md §8(e) mode 2) ----
#
# Every rank receives the same keys (the caller's batch) and reads them against
# its own shard on its own GPU: lookup + gather + decode (ResidentTable), so a
# key it does not own is a miss -- an all-null row, zero bytes in every buffer
# (arrow-rs null slots are zero, validity bit 0, utf8 length 0).  A key lives in
# exactly one shard, so for every row at most one rank contributes non-zero
# bytes, and the caller-order result (src/io/store/rocksdb/mod.rs:368-399:
# output row i is key i) is the byte-wise SUM of the ranks' buffers.  That is
# the one exchange step of the read: fixed-width values, bool bitmaps and
# validity bitmaps are summed as u8 (disjoint bytes / bits, so no carries),
# utf8 lengths are summed, every rank places its strings at the merged
# offsets, and the string bytes are summed.  Three all-reduces per read, each
# over all projected columns at once (few, large collectives); on GPUs the
# buffers can stay in HBM and go over RCCL, on CPU (tests) gloo carries them.


def _bitmap(h, n):
    nb = (n + 7) // 8
    if h["validity"] is None:  # no nulls on this rank: every row valid here
        import numpy as np
        v = np.full(nb, 0xFF, np.uint8)
        if n % 8:
            v[-1] = (1 << (n % 8)) - 1
        return v
    import numpy as np
    return np.frombuffer(bytes(h["validity"][:nb]), np.uint8)


def merge_reads(group, dtypes, n: int, hs):
    """Merge this rank's host buffer dicts (one per requested column, caller
    order, misses all-null) with every other rank's: returns the dicts of the
    whole read.  `group` is a Group (world 1 returns the input unchanged)."""
    if group.dist is None:
        return hs
    import numpy as np
    import torch
    from .schema import DTypeName as D
    nb = (n + 7) // 8
    # 1. validity + fixed values + bool bitmaps + utf8 lengths: one u8 buffer
    parts, lens_parts = [], []
    for dt, h in zip(dtypes, hs):
        parts.append(_bitmap(h, n))
        if dt == D.Utf8:
            lens_parts.append(np.diff(np.asarray(h["offsets"], np.int64)))
        else:
            parts.append(np.frombuffer(bytes(h["values"]), np.uint8)[: (nb if dt == D.Bool else n * dt.size())])
    flat = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, np.uint8))
    group.dist.all_reduce(flat)
    lens = None
    if lens_parts:
        lens = torch.from_numpy(np.concatenate(lens_parts))
        group.dist.all_reduce(lens)
        lens = lens.numpy().reshape(len(lens_parts), n)
    flat = flat.numpy()
    # 2. utf8: merged offsets, this rank's strings placed there, summed
    goffs, data_parts, at, u = [], [], 0, 0
    for dt, h in zip(dtypes, hs):
        if dt != D.Utf8:
            continue
        go = np.zeros(n + 1, np.int64)
        np.cumsum(lens[u], out=go[1:])
        if go[-1] > np.iinfo(np.int32).max:
            from .errors import SegmentError
            raise SegmentError("byte array offset overflow")
        lo = np.asarray(h["offsets"], np.int64)
        mine = np.diff(lo)
        buf = np.zeros(int(go[-1]), np.uint8)
        rows = np.flatnonzero(mine)
        if rows.size:
            ln = mine[rows]
            src = np.repeat(lo[rows] - np.cumsum(ln) + ln, ln) + np.arange(int(ln.sum()))
            dst = np.repeat(go[rows] - np.cumsum(ln) + ln, ln) + np.arange(int(ln.sum()))
            buf[dst] = np.frombuffer(bytes(h["values"]), np.uint8)[src]
        goffs.append(go)
        data_parts.append(buf)
        u += 1
    if data_parts:
        data = torch.from_numpy(np.concatenate(data_parts))
        group.dist.all_reduce(data)
        data = data.numpy()
    # 3. unpack
    out, pos, dpos, u = [], 0, 0, 0
    for dt, h in zip(dtypes, hs):
        valid = flat[pos:pos + nb]
        pos += nb
        nulls = n - int(np.unpackbits(valid, bitorder="little")[:n].sum()) if n else 0
        r = {"dtype": int(dt), "length": n, "null_count": nulls,
             "validity": valid.tobytes() if nulls else None, "offsets": None}
        if dt == D.Utf8:
            go = goffs[u]
            r["offsets"] = go.astype(np.int32)
            r["values"] = data[dpos:dpos + int(go[-1])].tobytes()
            dpos += int(go[-1])
            u += 1
        else:
            w = nb if dt == D.Bool else n * dt.size()
            r["values"] = flat[pos:pos + w].tobytes()
            pos += w
        out.append(r)
    return out


class ShardedResidentTable:
    """One key-range shard of a table per rank (one process per GPU), each a
    ResidentTable in that GPU's HBM.  `read` is Table::read over the whole
    table: every rank passes the same keys and gets the same caller-order
    batch.

    Not the default multi-GPU read: every rank looks up every key and the
    ranks byte-sum their host results over the process group (merge_reads),
    which suits a job whose ranks all want the same batch (a data-parallel
    reader on gloo or RCCL).  A server that owns all of a node's GPUs reads
    through MultiDeviceTable (murr_multi_gather: lookups on each GPU at once,
    one caller-order block on the home GPU, no collective)."""

    def __init__(self, table, group: "Group", ctx=None, name: str = "shard"):
        from .resident import ResidentTable
        self.group = group
        self.local = ResidentTable(table, ctx, name)

    def write_shard(self, batch):
        """Write this rank's keys (Table::write on its own shard).  Every key
        must be this rank's (shard_of): a key on two ranks would break the
        byte-sum merge of reads (route a batch first with route_batch)."""
        if self.group.world > 1:
            key = self.local.t.table.key
            check_owned(batch.column(batch.schema.get_field_index(key)), self.group.rank, self.group.world)
        self.local.write(batch)

    def read(self, keys, columns):
        from .resident import host_batch
        req, hs = self.local.read_host(keys, columns)
        merged = merge_reads(self.group, [c.dtype for c in req], len(keys), hs)
        return host_batch(req, merged)
