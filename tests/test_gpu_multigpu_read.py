"""murr_multi_gather, the read path of MultiDeviceTable: the shards' lookups
enqueued on their own streams, the caller-order block built on the home
stream after event waits (no host round trip), both the one-call form and
the two-phase form (sizes first, then murr_multi_gather_copy), at read sizes
whose scan takes several groups.  Against the MemoryStore restatement of
the whole table (src/io/store/rocksdb/mod.rs:368-399)."""
import numpy as np
import pytest

import murr_amd.multigpu as MG
from murr_amd.device import Context, device_count
from murr_amd.multigpu import MultiDeviceTable

from test_gpu_resident import assert_same, batch_c, expected, schema_c

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def table8():
    ndev = device_count()
    ctxs = [Context(i % ndev) for i in range(8)]
    t = MultiDeviceTable(schema_c(), ctxs)
    b1 = batch_c(30000, seed=3)
    b2 = batch_c(5000, start=28000, seed=5)  # 2000 rewrites
    t.write(b1)
    t.write(b2)
    return t, [b1, b2]


@pytest.mark.parametrize("two_phase", [False, True])
@pytest.mark.parametrize("nq", [1, 4096, 4097, 20000])
def test_eight_shards_read(table8, monkeypatch, two_phase, nq):
    t, batches = table8
    if two_phase:
        monkeypatch.setattr(MG, "TWO_PHASE_BYTES", 0)
    rng = np.random.default_rng(nq)
    q = [f"key{int(x)}" for x in rng.integers(0, 34000, size=nq)]
    if nq > 10:
        q[:3] = ["absent", "key29999", "key29999"]
    cols = ["c11", "c0", "c12", "c5"]
    assert_same(t.read(q, cols), expected(batches, q, cols))


def test_longest_rows_of_skewed_table():
    """A read of only the longest rows of a table whose row sizes are skewed
    (a few 4 KiB strings among short rows): the decode's utf8 buffers must be
    sized for the gathered bytes, not for the table's mean row."""
    import pyarrow as pa
    ndev = device_count()
    t = MultiDeviceTable(schema_c(), [Context(i % ndev) for i in range(4)])
    b = batch_c(3000, seed=11)
    s = b.column("c12").to_pylist()
    long_keys = []
    for i in range(0, 3000, 97):
        s[i] = chr(ord("a") + i % 26) * 4096
        long_keys.append(f"key{i}")
    b = pa.RecordBatch.from_arrays([*b.columns[:13], pa.array(s, pa.string()), *b.columns[14:]],
                                   names=b.schema.names)
    t.write(b)
    for q in (long_keys[:1], long_keys, long_keys + ["absent", "key5"]):
        assert_same(t.read(q, ["c12", "c11", "c3"]), expected([b], q, ["c12", "c11", "c3"]))
