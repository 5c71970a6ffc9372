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


# ---- random-key batch read across shards (SURVEY.md §8(e) mode 2) -----------------
# Each rank "reads" only the caller's keys it owns against its own shard (here
# the oracle decodes a block of those keys, exactly what ResidentTable.read_host
# returns on a GPU), then gather_reads sends the rows to the home rank point to
# point, which restores the whole read in caller order.  It must equal the
# oracle's decode of the read against the whole table.
READ_ROWS, READ_KEYS = 3001, 1500


def _read_case():
    from randgen import ALL, random_columns
    rng = np.random.default_rng(77)
    dtypes = ALL + [O_UTF8_EXTRA]
    cols = random_columns(rng, dtypes, READ_ROWS, null_p=0.15)
    seg = O.Segment([int(d) for d in dtypes])
    blob, off = O.encode_batch(seg, synth.oracle_cols(cols), READ_ROWS)
    q = rng.integers(0, int(READ_ROWS * 1.05), size=READ_KEYS)  # ~5 % misses, duplicates
    proj = [0, 12, 3, 1, 10, 11, 9, 5, 0]
    return dtypes, seg, blob, off, q, proj


O_UTF8_EXTRA = 0  # a second utf8 column


def _block_for(blob, off, q):
    parts, ro = [], [0]
    for k in q:
        k = int(k)
        b = blob[int(off[k]):int(off[k + 1])].tobytes() if k < READ_ROWS else b""
        parts.append(b)
        ro.append(ro[-1] + len(b))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(ro, np.uint64)


def _owner(keys, world):
    """Key-range owners (a key past the table: the last rank, where it misses)."""
    own = np.full(len(keys), world - 1, np.int64)
    for r in range(world):
        start, n = shard_rows(r, world, READ_ROWS)
        own[(keys >= start) & (keys < start + n)] = r
    return own


def _read_worker(rank, world, port, home, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from murr_amd.schema import DTypeName as D
    from murr_amd.shard import gather_reads
    g = Group("gloo")
    dtypes, seg, blob, off, keys, proj = _read_case()
    owner = _owner(keys, world)
    data, ro = _block_for(blob, off, keys[owner == rank])  # this rank's keys only
    local = O.decode_block(seg, proj, data, ro)
    merged = gather_reads(g, [D(dtypes[p]) for p in proj], len(keys), owner, local, home)
    q.put((rank, None if merged is None else
           [(m["null_count"], m["validity"], m["values"], None if m["offsets"] is None else m["offsets"].tolist())
            for m in merged]))
    g.close()


@pytest.mark.parametrize("world,home", [(2, 0), (3, 0), (3, 2)])
def test_sharded_random_key_read_restores_caller_order(world, home):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_read_worker, args=(r, world, port, home, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] is None for r in range(world) if r != home)  # only the home rank holds the read
    dtypes, seg, blob, off, keys, proj = _read_case()
    data, ro = _block_for(blob, off, keys)
    want = O.decode_block(seg, proj, data, ro)
    nb = (len(keys) + 7) // 8
    for p, (nulls, validity, values, offsets) in enumerate(got[home]):
        w = want[p]
        assert nulls == w["null_count"], p
        assert (validity is None) == (w["validity"] is None), p
        if validity is not None:
            assert validity[:nb] == w["validity"], p
        assert values == w["values"], p
        if w["offsets"] is not None:
            assert offsets == w["offsets"].tolist(), p


def test_pack_rows_round_trip():
    # one rank's packed rows unpack to the same cells (every dtype, nulls,
    # empty strings, zero rows)
    from murr_amd.schema import DTypeName as D
    from murr_amd.shard import _unpack_rows, pack_rows
    dtypes, seg, blob, off, keys, proj = _read_case()
    for m in (0, 1, 9, 700):
        data, ro = _block_for(blob, off, keys[:m])
        hs = O.decode_block(seg, proj, data, ro)
        dts = [D(dtypes[p]) for p in proj]
        cols = _unpack_rows(dts, m, pack_rows(dts, m, hs))
        for dt, h, (valid, payload) in zip(dts, hs, cols):
            nulls = m - int(valid.sum())
            assert nulls == h["null_count"]
            if dt == D.Utf8:
                lens, src = payload
                assert lens.tolist() == np.diff(h["offsets"].astype(np.int64)).tolist()
                assert src.tobytes() == h["values"]


# ---- key routing (murr_shard_of) -----------------------------------------------------

def _shard_of_py(key: bytes, n: int) -> int:
    """Restatement of murr_shard_of: fmix64(FNV-1a 64) mod n."""
    m = (1 << 64) - 1
    h = 0xcbf29ce484222325
    for b in key:
        h = ((h ^ b) * 0x100000001b3) & m
    h ^= h >> 33
    h = (h * 0xff51afd7ed558ccd) & m
    h ^= h >> 33
    h = (h * 0xc4ceb9fe1a85ec53) & m
    h ^= h >> 33
    return h % n


def test_shard_of_matches_restatement_and_balances():
    import pyarrow as pa
    from murr_amd.shard import shard_of
    keys = [f"key{i}" for i in range(20000)] + ["", "é", "a" * 300]
    for n in (1, 2, 3, 8):
        got = shard_of(keys, n)
        assert got.tolist() == [_shard_of_py(k.encode(), n) for k in keys]
        if n > 1:
            counts = np.bincount(got, minlength=n)
            assert counts.min() > 0.9 * len(keys) / n  # balanced
    # arrays with an offset, string or binary, give the same owners
    arr = pa.array(keys, pa.string()).slice(5, 100)
    assert shard_of(arr, 8).tolist() == shard_of(keys[5:105], 8).tolist()


def test_route_batch_and_owned_check():
    import pyarrow as pa
    from murr_amd.shard import check_owned, route_batch, shard_of
    keys = [f"k{i}" for i in range(5000)] + ["k7", "k7"]  # a repeated key lands on one shard
    batch = pa.RecordBatch.from_arrays([pa.array(keys), pa.array(np.arange(len(keys)))], names=["key", "v"])
    parts = route_batch(batch, "key", 3)
    assert sum(p.num_rows for p in parts) == batch.num_rows
    for r, p in enumerate(parts):
        check_owned(p.column(0), r, 3)
        assert p.column(1).to_pylist() == sorted(p.column(1).to_pylist())  # order kept
    owners = {k: int(o) for k, o in zip(keys, shard_of(keys, 3))}
    assert sum(1 for p in parts if "k7" in p.column(0).to_pylist()) == 1
    other = (owners["k7"] + 1) % 3
    with pytest.raises(ValueError, match="belong to other shards"):
        check_owned(pa.array(["k7"]), other, 3)


def _bench(*argv, timeout=180):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=timeout, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_spawns_its_own_ranks():
    # `bench.py --gpus N` without torchrun starts N rank processes itself; the
    # harness self-test mode runs the same spawner / barrier / max-sum / JSON
    # path with a host copy as the step (no GPU here)
    rc, line, err = _bench("--mode", "harness", "--gpus", "2", "--steps", "3", "--warmup", "1")
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["data"] == "harness self-test"
    assert line["scaling"] == "weak" and line["value"] > 0


def test_bench_refuses_ranks_without_gpus():
    # a decode run with more ranks than GPUs exits non-zero instead of sharing
    rc, line, err = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu")
    assert rc != 0 and line is None


def test_bench_table_split_over_ranks():
    # configs[3] as written: ONE table of --table-rows rows split by key range
    # over the ranks (strong scaling), through the spawner in harness mode
    rc, line, err = _bench("--mode", "harness", "--config", "D", "--table-rows", "10000001", "--gpus", "2",
                           "--steps", "2", "--warmup", "1")
    assert rc == 0, err[-2000:]
    cfg = line["config"]
    assert line["scaling"] == "strong" and line["n_gpus"] == 2
    assert cfg["table_rows"] == 10000001 and cfg["rows_per_rank"] == [5000001, 5000000]
    assert cfg["rows_summed_over_ranks"] == 10000001
