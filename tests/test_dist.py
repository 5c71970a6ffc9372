"""Multi-process (world size 2, gloo, CPU) rehearsal of the sharded path
(DESIGN.md §5): each rank owns a contiguous key range,
encodes and decodes only its shard (here with the CPU oracle: no GPU in this
container), and torch.distributed carries only the barrier and the
max/sum reductions bench.py reports.  The shards' decoded outputs must
concatenate to the single-process decode of the whole key range."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

import oracle as O  # noqa: E402
from murr_amd import synth  # noqa: E402
from murr_amd.shard import Group, shard_rows  # noqa: E402

TOTAL = 5003


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _decode_range(start, n):
    cols = synth.config_b(n, start=start)
    seg = O.Segment([int(c["dtype"]) for c in cols])
    blob, off = O.encode_batch(seg, synth.oracle_cols(cols), n)
    return O.decode_block(seg, [0, 1], blob, off), int(blob.size)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    g = Group("gloo")
    assert g.world == world and g.rank == rank
    start, n = shard_rows(rank, world, TOTAL)
    g.barrier()
    res, blob_bytes = _decode_range(start, n)
    g.barrier()
    strings = res[1]
    total_bytes = g.sum(float(blob_bytes))
    slowest = g.max(float(rank + 1))
    q.put((rank, start, n, strings["offsets"].tolist(), strings["values"], total_bytes, slowest))
    g.close()


def test_shard_rows_partition():
    for total in (0, 1, 7, 5003, 10_000_000):
        for world in (1, 2, 3, 8):
            spans = [shard_rows(r, world, total) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(n for _, n in spans) == total
            for (s0, n0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + n0 == s1
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1
    with pytest.raises(ValueError):
        shard_rows(2, 2, 10)


def test_group_world_one_is_identity(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    g = Group()
    assert g.world == 1 and g.rank == 0
    assert g.max(3.5) == 3.5 and g.sum(2.0) == 2.0
    g.barrier()
    g.close()


def test_two_rank_shards_concatenate_to_whole():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole_bytes = 0
    # key-range shards in rank order == one decode of the whole range, string by string
    offs_all, vals_all = [0], b""
    for rank, start, n, offs, vals, total_bytes, slowest in got:
        assert slowest == 2.0
        offs = np.asarray(offs, dtype=np.int64)
        offs_all.extend((offs[1:] + len(vals_all)).tolist())
        vals_all += vals
        whole_bytes = total_bytes
    ref, ref_blob = _decode_range(0, TOTAL)
    assert offs_all == ref[1]["offsets"].tolist()
    assert vals_all == ref[1]["values"]
    assert whole_bytes == ref_blob  # sum over ranks of shard blob bytes == whole-range blob
