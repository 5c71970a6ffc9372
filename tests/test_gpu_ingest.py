"""Ingest -> encode on the device -> read back.

The reference's own data file (util/example.parquet, tests/golden/example.parquet)
goes through the write handler's body parsing (src/api/http/handlers.rs:132-141)
into Table::write: the blobs the device encode writes are the oracle's blobs
for the same columns, and a device-resident read of every key returned as an
IPC stream re-ingests to the original table."""
import os

import numpy as np
import pyarrow as pa
import pytest

import oracle as O
from murr_amd import ColumnSchema, TableSchema, ingest, synth
from murr_amd.resident import ResidentTable
from murr_amd.schema import DTypeName as D
from murr_amd.store import MemoryStore
from murr_amd.table import Table

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SCHEMA = TableSchema("key", {"key": ColumnSchema(D.Utf8, False), "value": ColumnSchema(D.Int64)})


def body():
    with open(os.path.join(GOLDEN, "example.parquet"), "rb") as f:
        return f.read()


def test_parquet_ingest_blobs_match_oracle():
    t = Table.create(MemoryStore(), "ex", SCHEMA)
    batch = ingest.batch_from_body(body(), ingest.PARQUET_MIME)
    keys, blob, offs = t.encode(batch)
    v = batch.column("value")
    col = synth.column(D.Int64, np.asarray(v.fill_null(0), dtype=np.int64), ~np.asarray(v.is_null()))
    want_blob, want_off = O.encode_batch(O.Segment([int(D.Int64)]), synth.oracle_cols([col]), batch.num_rows)
    assert offs.tolist() == want_off.tolist()
    assert blob.tobytes() == want_blob.tobytes()
    assert ingest.write_body(t, body(), ingest.PARQUET_MIME) == batch.num_rows
    ks = keys.to_pylist()
    out = t.read(ks[::-1] + ["nope"], ["value"])
    assert out.column(0).to_pylist() == v.to_pylist()[::-1] + [None]


def test_parquet_to_resident_to_ipc_roundtrip():
    rt = ResidentTable(SCHEMA)
    n = ingest.write_body(rt, body(), ingest.PARQUET_MIME)
    src = ingest.batch_from_body(body(), ingest.PARQUET_MIME)
    keys = src.column("key").to_pylist()
    rng = np.random.default_rng(3)
    order = rng.permutation(n)
    q = [keys[i] for i in order]
    stream = rt.read_ipc(q, ["value"])
    back = ingest.batch_from_body(stream, ingest.ARROW_IPC_MIME)
    assert back.num_rows == n
    assert back.column(0).to_pylist() == [src.column("value")[int(i)].as_py() for i in order]
