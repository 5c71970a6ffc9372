"""MultiDeviceTable: mode-2 reads across key-owned shards without a collective
(murr_amd/multigpu.py): rows routed by murr_shard_of, gathered on their
shard's GPU, peer-copied to the home GPU, put in caller order by one gather
and decoded once.  The result must equal the MemoryStore restatement of the
whole table: caller order, misses as all-null rows, duplicates, later writes
winning (src/io/store/rocksdb/mod.rs:368-399, src/io/store/memory.rs:47-60).
The box has one GPU, so the shards are contexts on device 0 (the peer copy
is then a device copy); on an 8-GPU node each shard is its own device."""
import numpy as np
import pyarrow as pa
import pytest

from murr_amd.device import Context, device_count
from murr_amd.multigpu import MultiDeviceTable

from test_gpu_resident import C_DTYPES, assert_same, batch_c, expected, schema_c

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nshards", [1, 3])
def test_multi_device_reads_equal_whole_table(nshards):
    ndev = device_count()
    ctxs = [Context(i % ndev) for i in range(nshards)]
    t = MultiDeviceTable(schema_c(), ctxs)
    rng = np.random.default_rng(11 + nshards)
    b1 = batch_c(4000, seed=1)
    keys2 = [f"key{i}" for i in range(3000, 6000)]  # 1000 rewrites, 2000 new keys
    b2 = batch_c(3000, start=3000, seed=2, keys=keys2)
    t.write(b1)
    t.write(b2)
    q = [f"key{int(x)}" for x in rng.integers(0, 6300, size=2500)] + ["key3500"] * 3 + ["nope", ""]
    for cols in ([f"c{i}" for i in range(len(C_DTYPES))], ["c12", "c0", "c12"], ["c11"]):
        assert_same(t.read(q, cols), expected([b1, b2], q, cols))
    # every key lives on exactly one shard
    total = sum(sh.n for sh in t.shards)
    assert total == b1.num_rows + b2.num_rows


def test_multi_device_empty_shards_and_all_miss():
    ctxs = [Context(0) for _ in range(4)]
    t = MultiDeviceTable(schema_c(), ctxs)
    b = batch_c(3, seed=4)  # 3 rows: at least one shard stays empty
    t.write(b)
    q = ["key0", "missing", "key2", "key1", "zz"]
    cols = ["c3", "c11"]
    assert_same(t.read(q, cols), expected([b], q, cols))
    assert_same(t.read(["x", "y"], cols), expected([b], ["x", "y"], cols))
