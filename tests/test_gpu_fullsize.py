"""BASELINE.json sizes through size-independent properties: encode -> decode is
the identity on Arrow buffers, the device encode equals the oracle / the closed
form, and a 1000-key random read equals the oracle.  (configs A, B, C/D, E)"""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal
from murr_amd import synth
from murr_amd.device import set_default_opts, Context, DeviceBlock, decode_blocks, download_array, encode_batch
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    """Decode through both kernels: run-time specialised and generic."""
    set_default_opts(kernel=request.param)
    yield request.param
    set_default_opts()


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def seg_of(dtypes):
    return SegmentSchema([(f"c{i}", D(int(d))) for i, d in enumerate(dtypes)])


def as_expected(c):
    """Arrow column (synth) -> buffer dict in the decode output convention."""
    n = c["n"]
    dt = int(c["dtype"])
    out = {"dtype": dt, "length": n, "offsets": None}
    if c["validity"] is not None:
        bits = np.unpackbits(c["validity"], bitorder="little")[:n]
        out["null_count"] = int(n - bits.sum())
        out["validity"] = np.packbits(bits, bitorder="little").tobytes() if out["null_count"] else None
    else:
        out["null_count"], out["validity"] = 0, None
    if dt == 0:
        out["offsets"] = c["offsets"] - c["offsets"][0]
        out["values"] = c["values"][c["offsets"][0]:c["offsets"][-1]].tobytes()
    elif dt == 1:
        v = np.unpackbits(c["values"], bitorder="little")[:n]
        if c["validity"] is not None:
            v = v & np.unpackbits(c["validity"], bitorder="little")[:n]
        out["values"] = np.packbits(v, bitorder="little").tobytes()
    else:
        out["values"] = c["values"].tobytes()
    return out


def roundtrip(ctx, cols, n, check_oracle_encode=True):
    dtypes = [c["dtype"] for c in cols]
    seg = seg_of(dtypes)
    blob, row_off, blen = encode_batch(ctx, seg, synth.upload_columns(ctx, cols), n)
    if check_oracle_encode:
        wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
        assert blen == wblob.size
        assert np.array_equal(row_off.download((n + 1) * 8).view(np.uint64), woff)
        assert blob.download(blen).tobytes() == wblob.tobytes()
    blk = DeviceBlock(blob, row_off, n, blen)
    proj = list(range(len(cols)))
    outs = decode_blocks(ctx, seg, proj, [blk])
    for p, c in enumerate(cols):
        got = download_array(ctx, outs.array(0, p), int(c["dtype"]), n)
        assert_array_equal(got, as_expected(c), f"column {p}")
    return seg, blob, row_off, blen


def test_config_a_1k_rows_single_f32(ctx):
    # configs[0]: benches/read_plain.rs's plumbing size, one f32 column, f = i;
    # device decode and the host path (pinned H2D -> decode -> D2H) through
    # ReadBatchBuilder, both against the oracle and the closed form
    import pyarrow as pa
    from murr_amd.row import ReadBatchBuilder
    cols = synth.config_a(1000)
    seg, blob, row_off, blen = roundtrip(ctx, cols, 1000)
    host_blob = blob.download(blen).tobytes()
    offs = row_off.download(8 * 1001).view(np.uint64)
    b = ReadBatchBuilder(seg, seg.columns, 1000, ctx)
    for i in range(1000):
        b.add_row(host_blob[offs[i]:offs[i + 1]])
    rb = b.build()
    assert rb.column(0).equals(pa.array(np.arange(1000, dtype=np.float32)))
    want = O.decode_block(O.Segment([int(D.Float32)]), [0], np.frombuffer(host_blob, np.uint8), offs)
    assert want[0]["values"] == rb.column(0).buffers()[1].to_pybytes()[:4000]


def test_config_b_100k_rows(ctx):
    roundtrip(ctx, synth.config_b(100_000), 100_000)
    roundtrip(ctx, synth.config_b(100_000, null_frac=0.1), 100_000)


def test_config_d_shard_1_25m_rows_16_cols(ctx):
    n = 1_250_000
    cols = synth.config_c(n, start=n)  # shard 1 of 8 (rows [1.25M, 2.5M))
    seg, blob, row_off, blen = roundtrip(ctx, cols, n)
    # config C read: 1000 random keys (~5 % misses) x 16 columns, vs the oracle
    rng = np.random.default_rng(44)
    keys = rng.integers(0, int(n * 1.05), size=1000)
    host = blob.download(blen)
    off = row_off.download((n + 1) * 8).view(np.uint64)
    parts, roff = [], [0]
    for k in keys:
        b = host[int(off[k]):int(off[k + 1])].tobytes() if k < n else b""
        parts.append(b)
        roff.append(roff[-1] + len(b))
    data = np.frombuffer(b"".join(parts), np.uint8).copy()
    roff = np.array(roff, np.uint64)
    proj = list(range(16))
    outs = decode_blocks(ctx, seg, proj, [DeviceBlock.upload(ctx, data, roff)])
    want = O.decode_block(O.Segment([int(c["dtype"]) for c in cols]), proj, data, roff)
    for p in proj:
        got = download_array(ctx, outs.array(0, p), int(cols[p]["dtype"]), 1000)
        assert_array_equal(got, want[p], f"col {p}")


def test_config_e_20m_rows_encode_closed_form(ctx):
    n = 20_000_000
    cols = synth.config_e(n)
    seg = seg_of([D.Float32] * 10)
    blob, row_off, blen = encode_batch(ctx, seg, synth.upload_columns(ctx, cols), n)
    assert blen == 42 * n
    rec = np.zeros(n, dtype=[("b0", "u1"), ("b1", "u1")] + [(f"c{i}", "<f4") for i in range(10)])
    rec["b0"], rec["b1"] = 0x00, 0xFC  # WriteRow 0xFF bitset with bits 0..9 cleared
    v = np.arange(n, dtype=np.float32)
    for i in range(10):
        rec[f"c{i}"] = v
    host = blob.download(blen)
    assert host.tobytes() == rec.tobytes()
    off = row_off.download((n + 1) * 8).view(np.uint64)
    assert np.array_equal(off, np.arange(n + 1, dtype=np.uint64) * 42)
    del rec, host
    outs = decode_blocks(ctx, seg, list(range(10)), [DeviceBlock(blob, row_off, n, blen)])
    for p in range(10):
        a = outs.array(0, p)
        assert a.null_count == 0
        got = download_array(ctx, a, 10, n)
        assert got["values"] == v.tobytes()
