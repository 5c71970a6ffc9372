"""Arrow IPC framing (murr_ipc_*).

The reference ends a read in arrow-rs's StreamWriter (src/api/http/handlers.rs:93-101)
or FlightDataEncoder (src/api/flight/mod.rs:85-87).  Checks, on the oracle's
decode of seeded blocks (all 12 dtypes, nulls, missing keys):
* pyarrow reads our stream back to the oracle's arrays, buffer for buffer;
* at alignment 8 our record-batch body is byte-identical to the body pyarrow's
  own IPC writer produces for the same arrays (Arrow C++ uses 8-byte padding);
* at alignment 64 (arrow-rs IpcWriteOptions::default) every buffer offset is a
  multiple of 64 and the padding is zero.
The host framing is pure host code (no GPU); the device packing tests are in
tests/test_gpu_ipc.py.
"""
import ctypes as C

import numpy as np
import pyarrow as pa
import pytest

import oracle as O
from randgen import ALL, drop_rows, random_columns
from murr_amd import _abi, ipc, synth
from murr_amd.errors import MurrError
from murr_amd.schema import DTypeName as D, SegmentSchema


def seg_of(dtypes):
    return SegmentSchema([(f"c{i}_{D(d).name.lower()}", D(d)) for i, d in enumerate(dtypes)])


def oracle_block(dtypes, n, seed, null_p=0.1, miss=()):
    rng = np.random.default_rng(seed)
    cols = random_columns(rng, dtypes, n, null_p=null_p)
    oseg = O.Segment([int(d) for d in dtypes])
    blob, row_off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    if miss:
        blob, row_off = drop_rows(blob, row_off, set(miss))
    return oseg, blob, row_off


class HostArrays:
    """murr_host_array_t[] over the oracle's decoded buffers (kept alive here)."""

    def __init__(self, arrays):
        self.keep = []
        self.c = (_abi.HostArray * max(len(arrays), 1))()
        for p, a in enumerate(arrays):
            h = self.c[p]
            h.length, h.null_count, h.dtype = a["length"], a["null_count"], a["dtype"]
            h.values = self._ptr(a["values"])
            h.values_len = len(a["values"])
            h.validity = self._ptr(a["validity"]) if a["validity"] is not None else None
            h.offsets = self._ptr(a["offsets"].tobytes()) if a["offsets"] is not None else None

    def _ptr(self, b):
        buf = C.create_string_buffer(bytes(b), max(len(b), 1))
        self.keep.append(buf)
        return C.addressof(buf)


def to_pyarrow(a):
    n, dt = a["length"], D(a["dtype"])
    validity = pa.py_buffer(a["validity"]) if a["validity"] is not None else None
    if dt == D.Utf8:
        bufs = [validity, pa.py_buffer(a["offsets"].tobytes()), pa.py_buffer(a["values"])]
    else:
        bufs = [validity, pa.py_buffer(a["values"])]
    return pa.Array.from_buffers(dt.arrow_dtype(), n, bufs, null_count=a["null_count"])


def messages(stream_bytes):
    r = pa.ipc.MessageReader.open_stream(pa.BufferReader(stream_bytes))
    out = []
    while True:
        try:
            out.append(r.read_next_message())
        except StopIteration:
            return out


def host_stream(seg, proj, want, n, align):
    cols = [seg.columns[i] for i in proj]
    hs = HostArrays(want)
    return ipc.stream(ipc.schema_message(seg, cols, align), ipc.batch_message_host(seg, cols, hs.c, n, align))


def check_against(stream_bytes, seg, proj, want, n):
    """pyarrow reads the stream back to exactly the oracle's arrays."""
    rd = pa.ipc.open_stream(stream_bytes)
    sch = rd.schema
    assert [f.name for f in sch] == [seg.columns[i].name for i in proj]
    assert [f.type for f in sch] == [seg.columns[i].dtype.arrow_dtype() for i in proj]
    assert all(f.nullable for f in sch) and sch.metadata is None
    batches = list(rd)
    assert len(batches) == 1
    rb = batches[0]
    assert rb.num_rows == n
    for p, w in enumerate(want):
        got = rb.column(p)
        assert got.null_count == w["null_count"], p
        if w["dtype"] not in (int(D.Float32), int(D.Float64)):  # NaN != NaN; floats are checked by bytes
            assert got.equals(to_pyarrow(w)), p
        bufs = got.buffers()
        nb = (n + 7) // 8
        if w["null_count"]:
            assert bufs[0].to_pybytes()[:nb] == w["validity"], p
        else:
            assert bufs[0] is None or bufs[0].size == 0, p
        if w["dtype"] == int(D.Utf8):
            assert bufs[1].to_pybytes()[: 4 * (n + 1)] == w["offsets"].tobytes(), p
            assert bufs[2].to_pybytes()[: len(w["values"])] == w["values"], p
        else:
            assert bufs[1].to_pybytes()[: len(w["values"])] == w["values"], p


@pytest.mark.parametrize("n,seed,null_p", [(0, 1, 0.1), (1, 2, 0.1), (7, 3, 0.5), (64, 4, 0.0), (1000, 5, 0.1),
                                           (4099, 6, 0.3)])
@pytest.mark.parametrize("align", [8, 64])
def test_host_stream_roundtrip(n, seed, null_p, align):
    dtypes = ALL + [D.Utf8, D.Float32, D.Int64]
    miss = set(range(0, n, 13))
    oseg, blob, row_off = oracle_block(dtypes, n, seed, null_p, miss)
    seg = seg_of(dtypes)
    proj = [12, 0, 3, 1, 5, 9, 11, 2, 4, 6, 7, 8, 10, 13, 14, 0]  # duplicates allowed (read.rs:69-83)
    want = O.decode_block(oseg, proj, blob, row_off)
    s = host_stream(seg, proj, want, n, align)
    check_against(s, seg, proj, want, n)


@pytest.mark.parametrize("n,seed", [(1, 11), (100, 12), (3001, 13)])
def test_body_matches_pyarrow_writer(n, seed):
    """Alignment 8: our body == pyarrow's body for the same arrays, byte for byte."""
    dtypes = ALL
    oseg, blob, row_off = oracle_block(dtypes, n, seed, 0.2, set(range(1, n, 17)))
    seg = seg_of(dtypes)
    proj = list(range(len(dtypes)))
    want = O.decode_block(oseg, proj, blob, row_off)
    ours = messages(host_stream(seg, proj, want, n, 8))
    rb = pa.RecordBatch.from_arrays([to_pyarrow(w) for w in want], names=[seg.columns[i].name for i in proj])
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, rb.schema) as w:
        w.write_batch(rb)
    theirs = messages(sink.getvalue())
    assert [m.type for m in ours] == [m.type for m in theirs] == ["schema", "record batch"]
    assert ours[1].body.to_pybytes() == theirs[1].body.to_pybytes()
    assert ours[1].metadata_version == theirs[1].metadata_version
    # our schema message parses to the same schema pyarrow wrote
    assert pa.ipc.read_schema(ours[0]).equals(pa.ipc.read_schema(theirs[0]))


def test_alignment_64_layout():
    """arrow-rs default: message prefix + metadata and every buffer 64-aligned, zero padding."""
    n = 333
    dtypes = [D.Utf8, D.Bool, D.Int16, D.Float64]
    oseg, blob, row_off = oracle_block(dtypes, n, 21, 0.25)
    seg = seg_of(dtypes)
    proj = [0, 1, 2, 3]
    want = O.decode_block(oseg, proj, blob, row_off)
    hs = HostArrays(want)
    msg = ipc.batch_message_host(seg, [seg.columns[i] for i in proj], hs.c, n, 64)
    assert msg[:4] == b"\xff\xff\xff\xff"
    meta = int.from_bytes(msg[4:8], "little")
    assert (8 + meta) % 64 == 0 and len(msg) % 64 == 0
    m = messages(msg + ipc.eos())[0]
    body = m.body.to_pybytes()
    assert len(msg) == 8 + meta + len(body)
    # expected layout in IPC order (validity, [offsets], values) per field
    at = 0
    for w in want:
        parts = [w["validity"] or b""]
        if w["dtype"] == int(D.Utf8):
            parts.append(w["offsets"].tobytes())
        parts.append(w["values"])
        for b in parts:
            assert body[at:at + len(b)] == b
            pad = -len(b) % 64
            assert body[at + len(b):at + len(b) + pad] == bytes(pad)
            at += len(b) + pad
    assert at == len(body)


def test_schema_all_dtypes():
    seg = seg_of(ALL)
    msg = ipc.schema_message(seg, seg.columns, 64)
    assert len(msg) % 64 == 0
    sch = pa.ipc.read_schema(pa.py_buffer(msg))
    assert [f.type for f in sch] == [d.arrow_dtype() for d in ALL]
    assert [f.name for f in sch] == [c.name for c in seg.columns]


def test_eos_and_empty_stream():
    assert ipc.eos() == b"\xff\xff\xff\xff\x00\x00\x00\x00"
    seg = seg_of([D.Utf8])
    s = ipc.stream(ipc.schema_message(seg, seg.columns))
    rd = pa.ipc.open_stream(s)
    assert list(rd) == [] and rd.schema.names == ["c0_utf8"]


def test_errors():
    L = _abi.lib()
    seg = seg_of([D.Int32])
    n = C.c_uint64()
    pj = (C.c_uint32 * 1)(0)
    hs = (_abi.HostArray * 1)()
    hs[0].dtype, hs[0].length = int(D.Int32), 0
    # zero columns: RecordBatch::try_new error (read.rs:106-108)
    assert L.murr_ipc_batch_host(C.byref(seg.c), pj, 0, hs, 0, 64, None, 0, C.byref(n)) == _abi.E_ARROW
    # bad alignment
    assert L.murr_ipc_batch_host(C.byref(seg.c), pj, 1, hs, 0, 12, None, 0, C.byref(n)) == _abi.E_ARGUMENT
    # column out of range
    bad = (C.c_uint32 * 1)(3)
    assert L.murr_ipc_schema(C.byref(seg.c), bad, 1, None, 64, None, 0, C.byref(n)) == _abi.E_ARGUMENT
    # dtype mismatch between the array and the segment column
    hs[0].dtype = int(D.Int64)
    assert L.murr_ipc_batch_host(C.byref(seg.c), pj, 1, hs, 0, 64, None, 0, C.byref(n)) == _abi.E_DTYPE
    # capacity
    hs[0].dtype = int(D.Int32)
    assert L.murr_ipc_batch_host(C.byref(seg.c), pj, 1, hs, 0, 64, None, 0, C.byref(n)) == _abi.OK
    buf = C.create_string_buffer(int(n.value))
    assert L.murr_ipc_batch_host(C.byref(seg.c), pj, 1, hs, 0, 64, buf, n.value - 1, C.byref(n)) == _abi.E_CAPACITY
    with pytest.raises(MurrError):
        ipc.schema_message(seg, seg.columns, 7)
