"""Ingest front-end (murr_amd/ingest.py): the body handling of the HTTP write
handler (src/api/http/handlers.rs:111-150) on CPU, with the reference's own
data file util/example.parquet (tests/golden/example.parquet) as input."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import oracle as O
from test_ipc import HostArrays, oracle_block, seg_of
from murr_amd import ingest, ipc
from murr_amd.errors import TableError
from murr_amd.schema import DTypeName as D

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def example_bytes():
    with open(os.path.join(GOLDEN, "example.parquet"), "rb") as f:
        return f.read()


def test_example_parquet_body():
    b = ingest.batch_from_body(example_bytes(), ingest.PARQUET_MIME)
    t = pq.read_table(os.path.join(GOLDEN, "example.parquet"))
    assert b.num_rows == t.num_rows > 0
    assert b.schema.names == ["key", "value"]
    assert pa.Table.from_batches([b]).equals(t.combine_chunks())


def test_parquet_row_groups_concatenated():
    t = pa.table({"key": [f"k{i}" for i in range(1000)], "v": pa.array(np.arange(1000, dtype=np.float32))})
    sink = pa.BufferOutputStream()
    pq.write_table(t, sink, row_group_size=128)
    b = ingest.batch_from_body(sink.getvalue().to_pybytes(), "application/vnd.apache.parquet; x=1")
    assert b.num_rows == 1000 and pa.Table.from_batches([b]).equals(t)


def test_ipc_body_first_batch_only():
    b1 = pa.record_batch({"key": ["a", "b"], "v": [1, 2]})
    b2 = pa.record_batch({"key": ["c"], "v": [3]})
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, b1.schema) as w:
        w.write_batch(b1)
        w.write_batch(b2)
    got = ingest.batch_from_body(sink.getvalue().to_pybytes(), ingest.ARROW_IPC_MIME)
    assert got.equals(b1)


def test_errors():
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, pa.schema([("key", pa.string())])):
        pass
    with pytest.raises(TableError, match="empty Arrow IPC stream"):
        ingest.batch_from_body(sink.getvalue().to_pybytes(), ingest.ARROW_IPC_MIME)
    with pytest.raises(TableError, match="invalid Parquet"):
        ingest.batch_from_body(b"PAR1 not really", ingest.PARQUET_MIME)
    with pytest.raises(TableError):
        ingest.batch_from_body(b"{}", "application/json")


def test_our_ipc_stream_reingests():
    """A read's IPC stream (murr_ipc_*) is a valid write body."""
    dtypes = [D.Utf8, D.Int64, D.Float32, D.Bool]
    n = 777
    oseg, blob, row_off = oracle_block(dtypes, n, 31, 0.2)
    seg = seg_of(dtypes)
    proj = [0, 1, 2, 3]
    want = O.decode_block(oseg, proj, blob, row_off)
    hs = HostArrays(want)
    cols = [seg.columns[i] for i in proj]
    body = ipc.stream(ipc.schema_message(seg, cols), ipc.batch_message_host(seg, cols, hs.c, n, 64))
    got = ingest.batch_from_body(body, ingest.ARROW_IPC_MIME)
    assert got.num_rows == n and got.schema.names == [c.name for c in cols]
    assert got.column(0).to_pylist() == pa.ipc.open_stream(body).read_next_batch().column(0).to_pylist()
