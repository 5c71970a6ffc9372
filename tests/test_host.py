"""Host-side logic mirroring src/io/table/mod.rs + src/io/store/memory.rs that
runs before any device call: schema derivation, name resolution and the
reference's error cases.  CPU only."""
import pyarrow as pa
import pytest

from murr_amd import (ArrowError, ColumnSchema, DTypeName, SegmentError, TableAlreadyExists,
                      TableError, TableNotFound, TableSchema)
from murr_amd.schema import SegmentSchema, dtype_from_arrow
from murr_amd.store import KeyValue, MemoryStore
from murr_amd.table import Table


def schema_id_score():  # table/mod.rs:172-191
    return TableSchema("id", {"id": ColumnSchema(DTypeName.Utf8, False),
                              "score": ColumnSchema(DTypeName.Float32, True)})


def test_segment_from_table_drops_key_and_assigns_offsets():
    # src/io/schema.rs:33-54: key removed wherever it sits; offsets in IndexMap order
    ts = TableSchema("k", {"a": ColumnSchema("float64"), "k": ColumnSchema("utf8"),
                           "b": ColumnSchema("utf8"), "c": ColumnSchema("bool")})
    seg = SegmentSchema.from_table(ts)
    assert [(c.name, c.index, c.offset) for c in seg.columns] == [("a", 0, 0), ("b", 1, 8), ("c", 2, 12)]
    assert seg.capacity == 13 and seg.bitset_size == 1


def test_arrow_schema_carries_key_metadata():
    s = schema_id_score().to_arrow()  # schema.rs:56-68
    assert s.metadata == {b"key": b"id"}
    assert [f.name for f in s] == ["id", "score"]
    assert not s.field("id").nullable and s.field("score").nullable


def test_dtype_from_arrow():
    assert dtype_from_arrow(pa.float32()) == DTypeName.Float32
    with pytest.raises(SegmentError):
        dtype_from_arrow(pa.date32())  # schema.rs:86-89


def test_serde_names():
    assert DTypeName.parse("uint64") == DTypeName.UInt64
    assert DTypeName.Float32.serde_name == "float32"


def test_read_unknown_column_errors():  # table/mod.rs:351-359
    t = Table.create(MemoryStore(), "t", schema_id_score())
    with pytest.raises(SegmentError):
        t.read(["a"], ["nope"])


def test_read_key_column_errors():  # table/mod.rs:361-369
    t = Table.create(MemoryStore(), "t", schema_id_score())
    with pytest.raises(SegmentError):
        t.read(["a"], ["id"])


def test_write_with_null_key_errors():  # table/mod.rs:371-378
    t = Table.create(MemoryStore(), "t", schema_id_score())
    b = pa.RecordBatch.from_arrays([pa.array([None], pa.string()), pa.array([1.0], pa.float32())],
                                   names=["id", "score"])
    with pytest.raises(SegmentError):
        t.write(b)


def test_write_non_utf8_key_array_errors():  # table/mod.rs:73-79
    t = Table.create(MemoryStore(), "t", schema_id_score())
    b = pa.RecordBatch.from_arrays([pa.array([1], pa.int64()), pa.array([1.0], pa.float32())],
                                   names=["id", "score"])
    with pytest.raises(SegmentError):
        t.write(b)


def test_write_dtype_mismatch_errors():  # codec/mod.rs:96-106 make_decoder_rejects_dtype_mismatch
    t = Table.create(MemoryStore(), "t", schema_id_score())
    b = pa.RecordBatch.from_arrays([pa.array(["a"]), pa.array(["nope"])], names=["id", "score"])
    with pytest.raises(SegmentError):
        t.write(b)


def test_write_missing_column_is_arrow_error():  # table/mod.rs:55-64 index_of
    t = Table.create(MemoryStore(), "t", schema_id_score())
    b = pa.RecordBatch.from_arrays([pa.array(["a"])], names=["id"])
    with pytest.raises(ArrowError):
        t.write(b)


def test_create_duplicate_errors():  # table/mod.rs:478-485
    s = MemoryStore()
    Table.create(s, "t", schema_id_score())
    with pytest.raises(TableAlreadyExists):
        Table.create(s, "t", schema_id_score())


def test_non_utf8_key_rejected():  # table/mod.rs:487-505
    ts = TableSchema("id", {"id": ColumnSchema(DTypeName.Float32, False)})
    with pytest.raises(TableError):
        Table.create(MemoryStore(), "t", ts)


def test_memory_store_unknown_table():  # memory.rs:148-155
    with pytest.raises(TableNotFound):
        MemoryStore().write("nope", [KeyValue(b"x", b"y")])


def test_memory_store_manifest():  # memory.rs:165-171
    s = MemoryStore()
    s.create_table("users", schema_id_score())
    assert s.manifest().contains("users")
    assert s.manifest().schema("users") == schema_id_score()
