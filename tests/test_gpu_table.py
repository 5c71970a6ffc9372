"""The reference's own table / store tests (src/io/table/mod.rs:157-506,
src/io/store/memory.rs:71-165, src/io/store/rocksdb/mod.rs:368-424) over the
GPU path: Table.write encodes on the device, MemoryStore.read feeds a
GPU-batched ReadBatchBuilder."""
import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from murr_amd.device import set_default_opts

from golden_util import GOLDEN
from murr_amd import ColumnSchema, DTypeName as D, TableSchema
from murr_amd.row import ReadBatchBuilder
from murr_amd.schema import SegmentSchema
from murr_amd.store import KeyValue, MemoryStore
from murr_amd.table import Table

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    """Decode through both kernels: run-time specialised and generic."""
    set_default_opts(kernel=request.param)
    yield request.param
    set_default_opts()


def schema_id_score():
    return TableSchema("id", {"id": ColumnSchema(D.Utf8, False), "score": ColumnSchema(D.Float32)})


def batch_id_score(ids, scores):
    return pa.RecordBatch.from_arrays([pa.array(ids, pa.string()), pa.array(scores, pa.float32())],
                                      names=["id", "score"])


def test_roundtrip_writes_and_reads_back():  # table/mod.rs:230-246
    t = Table.create(MemoryStore(), "t", schema_id_score())
    t.write(batch_id_score(["a", "b", "c"], [1.0, None, 3.0]))
    out = t.read(["a", "b", "c"], ["score"])
    assert out.num_rows == 3
    assert out.column(0).to_pylist() == [1.0, None, 3.0]


def test_read_returns_columns_in_request_order():  # table/mod.rs:248-302
    ts = TableSchema("id", {"id": ColumnSchema(D.Utf8, False), "score": ColumnSchema(D.Float32),
                            "label": ColumnSchema(D.Utf8)})
    t = Table.create(MemoryStore(), "t", ts)
    t.write(pa.RecordBatch.from_arrays([pa.array(["a", "b"]), pa.array([1.0, 2.0], pa.float32()),
                                        pa.array(["x", "y"])], names=["id", "score", "label"]))
    out = t.read(["a", "b"], ["label", "score"])
    assert out.schema.names == ["label", "score"]
    out = t.read(["a", "b"], ["score", "label"])
    assert out.schema.names == ["score", "label"]
    assert out.column(1).to_pylist() == ["x", "y"]
    assert all(f.nullable for f in out.schema)  # read.rs:105 Field::new(.., true)


def test_read_subset_of_columns():  # table/mod.rs:304-314
    t = Table.create(MemoryStore(), "t", schema_id_score())
    t.write(batch_id_score(["a"], [1.5]))
    out = t.read(["a"], ["score"])
    assert out.num_columns == 1 and out.column(0).to_pylist() == [1.5]


def test_write_reorders_columns():  # table/mod.rs:316-336
    b = pa.RecordBatch.from_arrays([pa.array([7.0], pa.float32()), pa.array(["a"])], names=["score", "id"])
    t = Table.create(MemoryStore(), "t", schema_id_score())
    t.write(b)
    assert t.read(["a"], ["score"]).column(0).to_pylist() == [7.0]


def test_read_missing_keys_returns_nulls():  # table/mod.rs:338-349
    t = Table.create(MemoryStore(), "t", schema_id_score())
    t.write(batch_id_score(["a"], [1.0]))
    assert t.read(["a", "missing"], ["score"]).column(0).to_pylist() == [1.0, None]


def test_mixed_dtypes_roundtrip():  # table/mod.rs:380-462
    ts = TableSchema("id", {"id": ColumnSchema(D.Utf8, False), "f32": ColumnSchema(D.Float32),
                            "f64": ColumnSchema(D.Float64), "label": ColumnSchema(D.Utf8)})
    b = pa.RecordBatch.from_arrays([pa.array(["a", "b", "c"]), pa.array([1.5, None, -2.5], pa.float32()),
                                    pa.array([None, 2.0, 3.0]), pa.array(["x", None, "z"])],
                                   names=["id", "f32", "f64", "label"])
    t = Table.create(MemoryStore(), "t", ts)
    t.write(b)
    out = t.read(["a", "b", "c"], ["f32", "f64", "label"])
    assert out.column(0).to_pylist() == [1.5, None, -2.5]
    assert out.column(1).to_pylist() == [None, 2.0, 3.0]
    assert out.column(2).to_pylist() == ["x", None, "z"]


def test_create_then_open_roundtrip():  # table/mod.rs:464-476
    s = MemoryStore()
    t = Table.create(s, "t", schema_id_score())
    t.write(batch_id_score(["a"], [9.0]))
    t2 = Table.open(s, "t", schema_id_score())
    assert t2.read(["a"], ["score"]).column(0).to_pylist() == [9.0]


def payload_segment():  # src/io/store/test_util.rs:9-16
    return SegmentSchema([("payload", D.Utf8)])


def put(store, table, rows):  # test_util.rs:18-30 (WriteRow::write_dynamic per row)
    seg = payload_segment()
    ts = TableSchema("id", {"id": ColumnSchema(D.Utf8, False), "payload": ColumnSchema(D.Utf8)})
    t = Table.open(store, table, ts)
    keys, blob, offs = t.encode(pa.RecordBatch.from_arrays(
        [pa.array([k for k, _ in rows]), pa.array([v for _, v in rows], pa.binary()).cast(pa.string())],
        names=["id", "payload"]))
    raw = blob.tobytes()
    store.write(table, [KeyValue(k.encode(), raw[offs[i]:offs[i + 1]]) for i, (k, _) in enumerate(rows)])
    del seg


def fetch(store, table, keys):  # test_util.rs:32-51
    seg = payload_segment()
    b = ReadBatchBuilder(seg, seg.columns, len(keys))
    arr = store.read(table, keys, b).column(0)
    return [None if v is None else v.encode() for v in arr.to_pylist()]


def users_schema():
    return TableSchema("id", {"id": ColumnSchema(D.Utf8, False), "payload": ColumnSchema(D.Utf8)})


def test_store_round_trip():  # memory.rs:101-122
    s = MemoryStore()
    s.create_table("users", users_schema())
    put(s, "users", [("alice", b"a-payload"), ("bob", b"b-payload"), ("carol", b"c-payload")])
    assert fetch(s, "users", [b"alice", b"bob", b"carol"]) == [b"a-payload", b"b-payload", b"c-payload"]


def test_store_missing_key_yields_none():  # memory.rs:124-146, rocksdb/mod.rs:401-424
    s = MemoryStore()
    s.create_table("users", users_schema())
    put(s, "users", [("alice", b"a-payload"), ("carol", b"c-payload")])
    assert fetch(s, "users", [b"alice", b"bob", b"carol"]) == [b"a-payload", None, b"c-payload"]


def test_store_preserves_caller_key_order():  # rocksdb/mod.rs:368-399
    s = MemoryStore()
    s.create_table("users", users_schema())
    put(s, "users", [("alice", b"a"), ("bob", b"b"), ("carol", b"c"), ("dave", b"d")])
    got = fetch(s, "users", [b"dave", b"alice", b"zzz", b"carol", b"bob"])
    assert got == [b"d", b"a", None, b"c", b"b"]


def test_example_parquet_roundtrip():
    # util/example.parquet (reference data file): write then read every key back
    t = pq.read_table(f"{GOLDEN}/example.parquet")
    ts = TableSchema("key", {"key": ColumnSchema(D.Utf8, False), "value": ColumnSchema(D.Int64)})
    tab = Table.create(MemoryStore(), "ex", ts)
    tab.write(t.to_batches()[0] if t.num_rows == t.to_batches()[0].num_rows else t.combine_chunks().to_batches()[0])
    keys = t.column("key").to_pylist()
    out = tab.read(keys[::-1] + ["nope"], ["value"])
    assert out.column(0).to_pylist() == t.column("value").to_pylist()[::-1] + [None]


def test_builder_empty_projection_is_arrow_error():
    from murr_amd import ArrowError
    seg = payload_segment()
    b = ReadBatchBuilder(seg, [], 1)
    with pytest.raises(ArrowError):
        b.build()
