"""Sharding across GPUs.

Bulk decode (mode 1, bench.py): one process per GPU, each decoding its own
contiguous key range; no data-path collective.  torch.distributed (gloo, CPU
tensors) carries only the start/stop barriers and the max-over-ranks time /
sum-over-ranks bytes the bench reports: every output cell depends on exactly
one input row (src/io/row/read.rs:85-91) and the utf8 offset prefix is local
to a block.

Random-key reads (mode 2) across one process per GPU (`gather_reads`,
`ShardedResidentTable`): every rank reads only the caller's keys it owns
against its own shard, and sends those rows to the home rank point to point,
which scatters them into caller order -- no collective on the data path.  Writes
are routed by key (`shard_of`) and `write_shard` refuses keys this rank does
not own.  The one-process form of mode 2 (one process driving every GPU: keys
routed on the host, rows gathered on their shard's GPU, one peer-copy gather
to the caller's GPU) is `murr_amd.multigpu.MultiDeviceTable`.
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
# The caller's keys are known to every rank, and so is each key's owner
# (shard_of, or a key range).  Every rank reads only the keys it owns against
# its own shard on its own GPU (lookup + gather + decode: ResidentTable), so
# the ranks together decode the batch once.  Each rank other than the home
# rank then SENDS its rows -- every requested column's validity bits, values,
# or utf8 lengths and bytes, m rows packed into one byte buffer -- to the home
# rank, point to point; the home rank knows which caller positions each rank
# owns and scatters the rows back into caller order (the positional contract
# of src/io/store/rocksdb/mod.rs:368-399: output row i is key i).  Each row
# crosses the wire once: O(batch) bytes in total, no collective on the data
# path (round 4's form all-reduced zero-padded full batches from every rank:
# O(world x batch)).


def _valid_bits(h, m):
    """Validity of m rows as a bool array (no validity buffer: all valid)."""
    if h["validity"] is None:
        return np.ones(m, bool)
    return np.unpackbits(np.frombuffer(bytes(h["validity"]), np.uint8), bitorder="little")[:m].astype(bool)


def pack_rows(dtypes, m: int, hs) -> np.ndarray:
    """This rank's m decoded rows (host buffer dicts, one per requested
    column) as one u8 buffer: per column the validity bitmap, then its values
    (fixed: m x W bytes; bool: a bitmap; utf8: m i32 lengths, then the bytes)."""
    from .schema import DTypeName as D
    parts = []
    nb = (m + 7) // 8
    for dt, h in zip(dtypes, hs):
        parts.append(np.packbits(_valid_bits(h, m), bitorder="little"))
        if dt == D.Utf8:
            o = np.asarray(h["offsets"], np.int64)
            parts.append(np.diff(o).astype(np.int32).view(np.uint8))
            parts.append(np.frombuffer(bytes(h["values"]), np.uint8)[: int(o[-1]) - int(o[0])])
        elif dt == D.Bool:
            parts.append(np.frombuffer(bytes(h["values"]), np.uint8)[:nb])
        else:
            parts.append(np.frombuffer(bytes(h["values"]), np.uint8)[: m * dt.size()])
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)


def _unpack_rows(dtypes, m: int, buf: np.ndarray):
    """pack_rows' inverse: per column (valid bool[m], payload)."""
    from .schema import DTypeName as D
    out, pos, nb = [], 0, (m + 7) // 8
    for dt in dtypes:
        valid = np.unpackbits(buf[pos:pos + nb], bitorder="little")[:m].astype(bool)
        pos += nb
        if dt == D.Utf8:
            lens = buf[pos:pos + 4 * m].view(np.int32).astype(np.int64)
            pos += 4 * m
            tot = int(lens.sum())
            out.append((valid, (lens, buf[pos:pos + tot])))
            pos += tot
        elif dt == D.Bool:
            out.append((valid, np.unpackbits(buf[pos:pos + nb], bitorder="little")[:m].astype(bool)))
            pos += nb
        else:
            w = m * dt.size()
            out.append((valid, buf[pos:pos + w].reshape(m, dt.size())))
            pos += w
    return out


def gather_reads(group, dtypes, n: int, owner: np.ndarray, hs, home: int = 0):
    """Assemble one caller-order read of n keys on the `home` rank.  `owner`
    (every rank's copy is the same): the rank that owns caller key i; `hs`:
    this rank's host buffer dicts for ITS keys only, in caller order.  Ranks
    other than home send their packed rows to home (point to point) and get
    None; home returns the merged buffer dicts of the whole read.  World 1
    returns `hs` unchanged."""
    from .schema import DTypeName as D
    if group.dist is None:
        return hs
    import torch
    rank, world = group.rank, group.world
    owner = np.asarray(owner)
    if rank != home:
        buf = pack_rows(dtypes, int((owner == rank).sum()), hs)
        group.dist.send(torch.tensor([buf.size], dtype=torch.int64), dst=home)
        if buf.size:
            group.dist.send(torch.from_numpy(buf), dst=home)
        return None
    rows = {}
    for r in range(world):
        m = int((owner == r).sum())
        if r == home:
            rows[r] = _unpack_rows(dtypes, m, pack_rows(dtypes, m, hs))
            continue
        size = torch.zeros(1, dtype=torch.int64)
        group.dist.recv(size, src=r)
        buf = torch.zeros(int(size.item()), dtype=torch.uint8)
        if buf.numel():
            group.dist.recv(buf, src=r)
        rows[r] = _unpack_rows(dtypes, m, buf.numpy())
    where = {r: np.flatnonzero(owner == r) for r in range(world)}
    out = []
    for p, dt in enumerate(dtypes):
        valid = np.zeros(n, bool)
        for r, idx in where.items():
            valid[idx] = rows[r][p][0]
        nulls = int(n - valid.sum())
        res = {"dtype": int(dt), "length": n, "null_count": nulls,
               "validity": np.packbits(valid, bitorder="little").tobytes() if nulls else None, "offsets": None}
        if dt == D.Utf8:
            lens = np.zeros(n, np.int64)
            for r, idx in where.items():
                lens[idx] = rows[r][p][1][0]
            go = np.zeros(n + 1, np.int64)
            np.cumsum(lens, out=go[1:])
            if go[-1] > np.iinfo(np.int32).max:
                from .errors import SegmentError
                raise SegmentError("byte array offset overflow")
            data = np.zeros(int(go[-1]), np.uint8)
            for r, idx in where.items():
                ln, src = rows[r][p][1]
                if not src.size:
                    continue
                start = go[idx]  # each of rank r's rows lands at its caller position's offset
                pos = np.repeat(start - np.cumsum(ln) + ln, ln) + np.arange(int(ln.sum()))
                data[pos] = src
            res["offsets"] = go.astype(np.int32)
            res["values"] = data.tobytes()
        elif dt == D.Bool:
            bits = np.zeros(n, bool)
            for r, idx in where.items():
                bits[idx] = rows[r][p][1]
            res["values"] = np.packbits(bits, bitorder="little").tobytes()
        else:
            vals = np.zeros((n, dt.size()), np.uint8)
            for r, idx in where.items():
                vals[idx] = rows[r][p][1]
            res["values"] = vals.tobytes()
        out.append(res)
    return out


class ShardedResidentTable:
    """One key-range shard of a table per rank (one process per GPU), each a
    ResidentTable in that GPU's HBM.  `read` is Table::read over the whole
    table, a collective call: every rank passes the same keys, reads the keys
    its shard owns, and the home rank gets the caller-order batch (the other
    ranks get None) -- rows sent to it point to point (gather_reads).

    A server that owns all of a node's GPUs reads through MultiDeviceTable
    instead (murr_multi_gather: lookups on each GPU at once, one caller-order
    block on the home GPU by peer copies, one process)."""

    def __init__(self, table, group: "Group", ctx=None, name: str = "shard"):
        from .resident import ResidentTable
        self.group = group
        self.local = ResidentTable(table, ctx, name)

    def write_shard(self, batch):
        """Write this rank's keys (Table::write on its own shard).  Every key
        must be this rank's (shard_of): reads look a key up on its owner only
        (route a batch first with route_batch)."""
        if self.group.world > 1:
            key = self.local.t.table.key
            check_owned(batch.column(batch.schema.get_field_index(key)), self.group.rank, self.group.world)
        self.local.write(batch)

    def read(self, keys, columns, home: int = 0):
        from .resident import host_batch
        import pyarrow as pa
        if not isinstance(keys, pa.Array):
            keys = list(keys)
        # owners from the keys as given (shard_of takes an Arrow array: its
        # scalars would not survive list())
        owner = shard_of(keys, self.group.world) if self.group.world > 1 else np.zeros(len(keys), np.uint32)
        sel = np.flatnonzero(owner == self.group.rank)
        mine = keys.take(pa.array(sel, pa.int64())) if isinstance(keys, pa.Array) else [keys[i] for i in sel]
        req, hs = self.local.read_host(mine, columns)
        merged = gather_reads(self.group, [c.dtype for c in req], len(keys), owner, hs, home)
        return None if merged is None else host_batch(req, merged)
