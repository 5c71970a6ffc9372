"""Ingest front-end: Arrow IPC / Parquet request bodies -> the encode kernels
(SURVEY.md §8(f) rank 3).

Mirrors the body handling of the HTTP write handler
(src/api/http/handlers.rs:111-150): an Arrow IPC stream body contributes its
first record batch ("empty Arrow IPC stream" when it has none), a Parquet body
is read whole and its batches concatenated (`concat_batches`; failures are
TableError("invalid Parquet: ...")).  The batch then goes to Table::write --
here `Table.write` (host store, device encode through murr_encode_host) or
`ResidentTable.write` (device encode + device key index).  The body parsing is
host work done by pyarrow, as arrow-rs's readers do it in the reference; the
per-row encode loop it feeds is the GPU kernel.  The JSON body
(`WriteRequest::into_record_batch`, src/api/http/convert.rs:41-60) belongs to
the API layer and is out of scope.
"""
from __future__ import annotations

import pyarrow as pa

from .errors import TableError

ARROW_IPC_MIME = "application/vnd.apache.arrow.stream"  # handlers.rs:21
PARQUET_MIME = "application/vnd.apache.parquet"        # handlers.rs:22


def batch_from_ipc(body: bytes) -> pa.RecordBatch:
    """StreamReader::try_new + next() (handlers.rs:125-131)."""
    try:
        reader = pa.ipc.open_stream(pa.py_buffer(body))
        batch = reader.read_next_batch()
    except StopIteration:
        raise TableError("empty Arrow IPC stream") from None
    except (pa.ArrowInvalid, pa.ArrowIOError) as e:
        raise TableError(f"Arrow error: {e}") from None
    return batch


def batch_from_parquet(body: bytes) -> pa.RecordBatch:
    """ParquetRecordBatchReaderBuilder + concat_batches (handlers.rs:132-141)."""
    import pyarrow.parquet as pq
    try:
        pf = pq.ParquetFile(pa.BufferReader(body))
        batches = list(pf.iter_batches())
    except (pa.ArrowInvalid, pa.ArrowIOError, OSError) as e:
        raise TableError(f"invalid Parquet: {e}") from None
    if not batches:
        # concat of zero batches: an empty batch of the file's schema
        return pa.RecordBatch.from_pylist([], schema=pf.schema_arrow)
    if len(batches) == 1:
        return batches[0]
    return pa.Table.from_batches(batches).combine_chunks().to_batches()[0]


def batch_from_body(body: bytes, content_type: str) -> pa.RecordBatch:
    """Content-type dispatch of write_table (handlers.rs:117-145)."""
    if ARROW_IPC_MIME in content_type:
        return batch_from_ipc(body)
    if PARQUET_MIME in content_type:
        return batch_from_parquet(body)
    raise TableError(f"unsupported content type '{content_type}' (JSON bodies are out of scope)")


def write_body(table, body: bytes, content_type: str) -> int:
    """Parse the body and write it through the table's encode path; returns rows written."""
    batch = batch_from_body(body, content_type)
    table.write(batch)
    return batch.num_rows
