"""Arrow IPC messages packed on the device (murr_ipc_batch_device, murr_ipc.hip).

Parity: the device-packed record-batch message is byte-identical to the host
framing (murr_ipc_batch_host, itself pinned against pyarrow's IPC writer in
tests/test_ipc.py) of the oracle's decode of the same block, and pyarrow reads
it back to the oracle's arrays.  End to end, ResidentTable.read_ipc (lookup,
gather, decode and packing on the device) yields the same stream bytes as
Table.read_ipc over a MemoryStore (the builder path the HTTP fetch handler
mirrors, src/api/http/handlers.rs:88-101)."""
import numpy as np
import pyarrow as pa
import pytest

import oracle as O
from randgen import ALL
from test_ipc import HostArrays, check_against, oracle_block, seg_of
from murr_amd import ColumnSchema, TableSchema, ipc, synth
from murr_amd.device import Context, DeviceBlock, decode_blocks
from murr_amd.resident import ResidentTable
from murr_amd.schema import DTypeName as D
from murr_amd.store import MemoryStore
from murr_amd.table import Table

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def device_message(ctx, seg, proj, blob, row_off, align):
    blk = DeviceBlock.upload(ctx, blob, row_off)
    outs = decode_blocks(ctx, seg, proj, [blk])
    dev, n = ipc.batch_message_device(ctx, seg, proj, outs, 0, blk.n_rows, align)
    assert ctx.last_kernel() == "ipc_pack"
    return ipc.download_message(ctx, dev, n)


def assert_same_bytes(got, exp):
    assert len(got) == len(exp), (len(got), len(exp))
    if got != exp:
        a, b = np.frombuffer(got, np.uint8), np.frombuffer(exp, np.uint8)
        bad = np.flatnonzero(a != b)
        raise AssertionError(f"{bad.size} bytes differ, first at {bad[:8].tolist()}: "
                             f"got {a[bad[:8]].tolist()} want {b[bad[:8]].tolist()}; "
                             f"metadata {int.from_bytes(got[4:8], 'little') + 8} bytes")


@pytest.mark.parametrize("n,seed,null_p", [(1, 1, 0.1), (63, 2, 0.5), (1000, 3, 0.0), (4099, 4, 0.1),
                                           (20000, 5, 0.2)])
@pytest.mark.parametrize("align", [8, 64])
def test_device_message_equals_host_framing(ctx, n, seed, null_p, align):
    dtypes = ALL + [D.Utf8, D.Float32]
    oseg, blob, row_off = oracle_block(dtypes, n, seed, null_p, set(range(2, n, 11)))
    seg = seg_of(dtypes)
    proj = [0, 12, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 0]
    want = O.decode_block(oseg, proj, blob, row_off)
    got = device_message(ctx, seg, proj, blob, row_off, align)
    cols = [seg.columns[i] for i in proj]
    hs = HostArrays(want)  # owns the buffers the framing reads
    exp = ipc.batch_message_host(seg, cols, hs.c, n, align)
    assert_same_bytes(got, exp)
    check_against(ipc.stream(ipc.schema_message(seg, cols, align), got), seg, proj, want, n)


def test_device_message_config_b_block(ctx):
    """One full config B block (100k rows, f32 + utf8 key string)."""
    n = 100_000
    cols = synth.config_b(n)
    dtypes = [int(c["dtype"]) for c in cols]
    oseg = O.Segment(dtypes)
    blob, row_off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    seg = seg_of([D(d) for d in dtypes])
    proj = [0, 1]
    want = O.decode_block(oseg, proj, blob, row_off)
    got = device_message(ctx, seg, proj, blob, row_off, 64)
    hs = HostArrays(want)
    exp = ipc.batch_message_host(seg, [seg.columns[i] for i in proj], hs.c, n, 64)
    assert_same_bytes(got, exp)


def test_device_capacity_error(ctx):
    import ctypes as C
    from murr_amd import _abi
    dtypes = [D.Int32, D.Utf8]
    oseg, blob, row_off = oracle_block(dtypes, 100, 9)
    seg = seg_of(dtypes)
    blk = DeviceBlock.upload(ctx, blob, row_off)
    outs = decode_blocks(ctx, seg, [0, 1], [blk])
    pj = (C.c_uint32 * 2)(0, 1)
    n, err = C.c_uint64(), _abi.Error()
    assert ctx.L.murr_ipc_batch_device(ctx.h, C.byref(seg.c), pj, 2, outs.arrays, 100, 64, None, 0,
                                       C.byref(n), C.byref(err)) == _abi.OK
    small = ctx.alloc(int(n.value) - 64)
    assert ctx.L.murr_ipc_batch_device(ctx.h, C.byref(seg.c), pj, 2, outs.arrays, 100, 64, small.ptr,
                                       small.nbytes, C.byref(n), C.byref(err)) == _abi.E_CAPACITY
    assert err.required == n.value


C_DTYPES = [D.Bool, D.Int8, D.Int16, D.Int32, D.Int64, D.UInt8, D.UInt16, D.UInt32, D.UInt64,
            D.Float32, D.Float64, D.Utf8, D.Utf8, D.Float32, D.Float64, D.Int64]


def schema_c():
    cols = {"key": ColumnSchema(D.Utf8, False)}
    for i, d in enumerate(C_DTYPES):
        cols[f"c{i}"] = ColumnSchema(d)
    return TableSchema("key", cols)


@pytest.mark.parametrize("align", [8, 64])
def test_resident_read_ipc_equals_builder_path(align):
    ts = schema_c()
    cols = synth.config_c(5000)
    keys = pa.array([f"key{i}" for i in range(5000)])
    batch = pa.RecordBatch.from_arrays([keys] + [synth.to_arrow(c) for c in cols],
                                       names=["key"] + [f"c{i}" for i in range(16)])
    rt = ResidentTable(ts)
    rt.write(batch)
    mt = Table.create(MemoryStore(), "t", ts)
    mt.write(batch)
    rng = np.random.default_rng(8)
    q = [f"key{i}" for i in rng.integers(0, 5300, size=1000)]  # ~6% misses
    req = ["c11", "c0", "c3", "c12", "c9", "c11", "c15"]
    got = rt.read_ipc(q, req, align)
    assert got == mt.read_ipc(q, req, align)
    rb = pa.ipc.open_stream(got).read_all()
    assert rb.column_names == req
    want = mt.read(q, req)
    for a, b in zip(rb.columns, want.columns):
        a = a.combine_chunks()
        assert a.null_count == b.null_count
        if not pa.types.is_floating(a.type):
            assert a.equals(b)


def test_resident_read_ipc_all_miss():
    rt = ResidentTable(schema_c())
    got = pa.ipc.open_stream(rt.read_ipc(["a", "b"], ["c3", "c11"])).read_all()
    assert got.num_rows == 2 and all(c.null_count == 2 for c in got.columns)
