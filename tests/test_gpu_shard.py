"""Random-key batch read over key-range shards on GPUs (SURVEY.md §8(e) mode 2):
two ranks (gloo, both on device 0 of the one-GPU box, each with its own
context and shard in HBM) read the same keys, each only the keys it owns, and
send their rows to the home rank; ShardedResidentTable.read on the home rank
must equal one ResidentTable holding the whole table, buffer for buffer (the
other rank gets None)."""
import os
import socket

import numpy as np
import pyarrow as pa
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu
ROWS, KEYS = 6000, 2000
COLS = ["c11", "c0", "c3", "c12", "c9", "c11", "c15", "c1"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case():
    from test_gpu_resident import batch_c, schema_c
    batch = batch_c(ROWS, seed=5)
    rng = np.random.default_rng(6)
    keys = [f"key{i}" for i in rng.integers(0, int(ROWS * 1.05), size=KEYS)]
    return schema_c(), batch, keys


def _worker(rank, world, port, q, arrow_keys=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from murr_amd.shard import Group, ShardedResidentTable, route_batch
    g = Group("gloo")
    ts, batch, keys = _case()
    t = ShardedResidentTable(ts, g)
    t.write_shard(route_batch(batch, "key", world)[rank])  # keys go to their owner shard
    # (the keys also as a pyarrow array, as a Flight handler hands them over)
    rb = t.read(pa.array(keys, pa.string()) if arrow_keys else keys, COLS, home=1)
    if rb is None:
        q.put((rank, None))
    else:
        sink = pa.BufferOutputStream()
        with pa.ipc.new_stream(sink, rb.schema) as w:
            w.write_batch(rb)
        q.put((rank, sink.getvalue().to_pybytes()))
    g.close()


@pytest.mark.parametrize("arrow_keys", [False, True])
def test_two_shards_equal_whole_table(arrow_keys):
    from murr_amd.resident import ResidentTable
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, arrow_keys)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    ts, batch, keys = _case()
    whole = ResidentTable(ts)
    whole.write(batch)
    want = whole.read(keys, COLS)
    got = dict(got)
    assert got[0] is None and got[1] is not None  # the batch lands on the home rank only
    for rank, raw in [(1, got[1])]:
        rb = pa.ipc.open_stream(raw).read_next_batch()
        assert rb.schema.equals(want.schema)
        for a, b in zip(rb.columns, want.columns):
            assert a.null_count == b.null_count
            ba, bb = a.buffers(), b.buffers()
            for x, y in zip(ba[1:], bb[1:]):
                assert x.to_pybytes() == y.to_pybytes(), rank
