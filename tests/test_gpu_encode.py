"""HIP encode (murr_encode_batch, through the C ABI) against the oracle: row
blobs and row offsets bit-exact (WriteRow semantics incl. 0xFF bitset padding)."""
import numpy as np
import pytest

import oracle as O
from golden_util import block_from_rows, encode_inputs, load_cases
from randgen import ALL, random_columns
from murr_amd import synth
from murr_amd.device import set_default_opts, Context, encode_batch
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    """Every encode test runs on both kernels: run-time specialised
    (murr_jit_encode.hip) and generic (murr_kernels.hip)."""
    set_default_opts(encode_kernel=request.param)
    yield request.param
    set_default_opts()
CASES = load_cases()


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def seg_of(dtypes):
    return SegmentSchema([(f"c{i}", D.parse(d)) for i, d in enumerate(dtypes)])


def gpu_encode(ctx, dtypes, cols, n):
    dcols = synth.upload_columns(ctx, cols)
    blob, row_off, blen = encode_batch(ctx, seg_of(dtypes), dcols, n)
    return blob.download(blen), row_off.download((n + 1) * 8).view(np.uint64)


def as_cols(dtypes, inputs, n):
    cols = []
    for d, c in zip(dtypes, inputs):
        cc = {"dtype": D.parse(d), "n": n, "offset": 0, "validity": None, "offsets": None}
        cc["values"] = np.frombuffer(c["values"] or b"\0" * 16, np.uint8).copy()
        if c["validity"] is not None:
            cc["validity"] = np.frombuffer(c["validity"], np.uint8).copy()
        if c["offsets"] is not None:
            cc["offsets"] = np.asarray(c["offsets"], np.int32)
        cols.append(cc)
    return cols


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden(ctx, case):
    n = len(case["rows"])
    cols = as_cols(case["dtypes"], encode_inputs(case), n)
    blob, off = gpu_encode(ctx, case["dtypes"], cols, n)
    data, want_off = block_from_rows(case["encode_blobs"] or case["rows"])
    assert np.array_equal(off, want_off)
    assert blob.tobytes() == data.tobytes()


@pytest.mark.parametrize("seed,n", [(21, 1), (22, 64), (23, 255), (24, 256), (25, 257), (26, 3000),
                                    (27, 40000)])
def test_random_vs_oracle(ctx, seed, n):
    rng = np.random.default_rng(seed)
    dtypes = [D(int(d)) for d in rng.choice(ALL, size=int(rng.integers(1, 20)))]
    cols = random_columns(rng, dtypes, n, null_p=float(rng.choice([0.0, 0.1, 0.7])))
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff)
    assert blob.tobytes() == wblob.tobytes()


def test_fixed_width_only_rows(ctx):
    n = 5000
    cols = synth.config_e(n)
    blob, off = gpu_encode(ctx, [D.Float32] * 10, cols, n)
    wblob, woff = O.encode_batch(O.Segment([10] * 10), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_long_strings_take_the_hbm_path(ctx):
    rng = np.random.default_rng(31)
    dtypes = [D.Utf8, D.Int16, D.Utf8]
    n = 600
    cols = random_columns(rng, dtypes, n, null_p=0.1, long_every=29, long_len=60000)
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_tiles_over_a_small_stage(ctx):
    # short strings keep the mean blob small (an 8 KiB LDS stage per 256-row
    # tile), while a few tiles of 120-byte strings overflow it: those tiles go
    # straight to HBM, the rest through the stage
    n = 20_000
    rng = np.random.default_rng(33)
    lens = np.full(n, 3, np.int64)
    lens[2560:3072] = 120  # tiles 10 and 11
    lens[7000:7100] = 120  # part of tile 27
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(97, 123, size=int(offs[-1]), dtype=np.uint8)
    cols = [synth.column(D.Float32, np.arange(n, dtype=np.float32)),
            synth.column(D.Utf8, offsets=offs.astype(np.int32), data=data)]
    blob, off = gpu_encode(ctx, [D.Float32, D.Utf8], cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(D.Float32), int(D.Utf8)]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_sliced_arrow_inputs(ctx):
    # Arrow arrays with a non-zero offset (RecordBatch::slice, dataset.rs:73-80)
    rng = np.random.default_rng(32)
    dtypes = [D.Bool, D.Utf8, D.Int64, D.UInt8]
    full = 1000
    cols = random_columns(rng, dtypes, full, null_p=0.3)
    k, n = 37, 500
    for c in cols:
        c["offset"] = k
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_sliced_inputs_without_validity(ctx):
    # no utf8 validity buffer: tile totals come from the offsets inside the
    # scan (murr_jit_encode.hip sizes_inline), from a slice's offset
    rng = np.random.default_rng(34)
    dtypes = [D.Utf8, D.Float32, D.Utf8]
    full = 3000
    cols = random_columns(rng, dtypes, full, null_p=0.0)
    k, n = 129, 2600
    for c in cols:
        assert c["validity"] is None
        c["offset"] = k
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_inline_tile_totals_over_several_scan_groups(ctx):
    # 1.2 M rows = 4688 tiles: two 4096-tile scan groups on the inline path,
    # and a ragged last tile
    n = 1_200_000 + 77
    cols = synth.config_b(n)
    blob, off = gpu_encode(ctx, [D.Float32, D.Utf8], cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(D.Float32), int(D.Utf8)]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()


def test_empty_batch(ctx):
    dtypes = [D.Utf8, D.Float32]
    cols = random_columns(np.random.default_rng(0), dtypes, 0)
    blob, off = gpu_encode(ctx, dtypes, cols, 0)
    assert off.tolist() == [0] and blob.size == 0


def test_wide_schema_encode(ctx, kernel_mode):
    # 70 columns: a 9-byte bitset, every dtype at every field alignment
    rng = np.random.default_rng(78)
    dtypes = [D(int(d)) for d in rng.choice(ALL, size=70)]
    n = 900
    cols = random_columns(rng, dtypes, n, null_p=0.2, max_str=9)
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff)
    assert blob.tobytes() == wblob.tobytes()


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_bitmaps_not_on_a_dword(ctx, shift):
    # validity and bool bitmaps at device addresses that are not 4-byte
    # aligned (any C caller may pass such a pointer): the wave's bitmap
    # windows are read from the dword below and shifted by the misalignment
    from types import SimpleNamespace
    rng = np.random.default_rng(90 + shift)
    dtypes = [D.Bool, D.Int32, D.Utf8, D.Bool, D.Float64, D.Int8]
    n = 3000 + shift
    cols = random_columns(rng, dtypes, n, null_p=0.3)
    dcols = synth.upload_columns(ctx, cols)
    keep = []
    for c, d in zip(cols, dcols):
        for key in ("validity",) + (("values",) if c["dtype"] == D.Bool else ()):
            if c[key] is None:
                continue
            buf = ctx.upload(np.concatenate([np.full(shift, 0xA5, np.uint8), c[key]]))
            keep.append(buf)
            d[key] = SimpleNamespace(ptr=buf.ptr + shift)
    blob, row_off, blen = encode_batch(ctx, seg_of(dtypes), dcols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(row_off.download((n + 1) * 8).view(np.uint64), woff)
    assert blob.download(blen).tobytes() == wblob.tobytes()


def _utf8_with_null_bytes(rng, n, null_p, max_str=20):
    # Arrow lets a null slot span bytes (only the validity bit says null):
    # every other null string here keeps its bytes
    valid = rng.random(n) >= null_p
    lens = rng.integers(0, max_str + 1, size=n)
    lens[~valid & (np.arange(n) % 2 == 0)] = 0
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0x20, 0x7F, size=int(offs[-1]), dtype=np.uint8)
    return synth.column(D.Utf8, valid=valid, offsets=offs.astype(np.int32), data=data, n=n)


def test_null_strings_with_bytes_are_recounted(ctx, kernel_mode):
    # The JIT encode estimates utf8 tile sizes from the offsets and validity
    # popcounts (exact when null strings are empty); null strings spanning
    # bytes make the estimate off, the kernel reports it and the host
    # recounts with the sizes pass: the output is the oracle's either way
    rng = np.random.default_rng(95)
    dtypes = [D.Utf8, D.Int32, D.Utf8]
    n = 50_000 + 3
    cols = [_utf8_with_null_bytes(rng, n, 0.3), random_columns(rng, [D.Int32], n, null_p=0.2)[0],
            _utf8_with_null_bytes(rng, n, 0.5)]
    before = ctx.stats()["encode_recounts"]
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()
    assert ctx.stats()["encode_recounts"] - before == (1 if kernel_mode == "jit" else 0)


@pytest.mark.parametrize("k", [0, 5, 35])
def test_validity_estimates_exact_for_empty_nulls(ctx, k):
    # empty null strings (as Arrow writers leave them): the estimated tile
    # sizes are exact -- no recount -- over several scan groups, sliced
    rng = np.random.default_rng(96 + k)
    dtypes = [D.Utf8, D.Float64, D.Utf8, D.Bool]
    full = 1_100_000 + 41
    cols = random_columns(rng, dtypes, full, null_p=0.25, max_str=12, unicode=False)
    n = full - k
    for c in cols:
        c["offset"] = k
    before = ctx.stats()["encode_recounts"]
    blob, off = gpu_encode(ctx, dtypes, cols, n)
    wblob, woff = O.encode_batch(O.Segment([int(d) for d in dtypes]), synth.oracle_cols(cols), n)
    assert np.array_equal(off, woff) and blob.tobytes() == wblob.tobytes()
    assert ctx.stats()["encode_recounts"] == before
