"""HIP decode (murr_decode_blocks, through the C ABI) against the oracle and the
golden fixtures: bit-exact Arrow buffers, first-error parity."""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal, block_from_rows, expected_array, load_cases
from randgen import ALL, drop_rows, random_columns
from murr_amd import MurrError, SegmentError, synth
from murr_amd.device import set_default_opts, Context, DeviceBlock, decode_blocks, download_array
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu
CASES = load_cases()


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


KERNEL = {"jit": "murr_jit_decode", "generic": "decode_kernel"}


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    """Every decode test runs on both kernels: the run-time specialised one
    (murr_jit_kernel.hip) and the generic one (murr_decode.hip)."""
    set_default_opts(kernel=request.param)
    yield request.param
    set_default_opts()


def seg_of(dtypes):
    return SegmentSchema([(f"c{i}", D.parse(d)) for i, d in enumerate(dtypes)])


def gpu_decode(ctx, seg, proj, blocks):
    dblocks = [DeviceBlock.upload(ctx, d, o) for d, o in blocks]
    outs = decode_blocks(ctx, seg, proj, dblocks)
    res = []
    for b, blk in enumerate(dblocks):
        row = []
        for p, ci in enumerate(proj):
            row.append(download_array(ctx, outs.array(b, p), int(seg.columns[ci].dtype), blk.n_rows))
        res.append(row)
    return res


def check_padding(got, n):
    raw = got["validity_raw"]
    nb = (n + 7) // 8
    if got["validity"] is not None:  # null_count 0: no validity buffer (its bytes are unspecified)
        if n % 8:
            assert raw[nb - 1] >> (n % 8) == 0, "validity bits past n must be zero"
        assert all(x == 0 for x in raw[nb:]), "validity padding must be zero"
    if got["dtype"] == 1:
        vals = got["values"]
        if n % 8:
            assert vals[nb - 1] >> (n % 8) == 0
        assert all(x == 0 for x in vals[nb:])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden(ctx, case):
    seg = seg_of(case["dtypes"])
    data, row_off = block_from_rows(case["rows"])
    if case["expect_error"]:
        with pytest.raises(SegmentError, match="invalid utf8"):
            gpu_decode(ctx, seg, case["proj"], [(data, row_off)])
        return
    got = gpu_decode(ctx, seg, case["proj"], [(data, row_off)])[0]
    for p, e in enumerate(case["expected"]):
        assert_array_equal(got[p], expected_array(e), f"{case['name']} col {p}")
        check_padding(got[p], e["length"])


def oracle_block(seg_dtypes, cols, n, missing=()):
    oseg = O.Segment([int(d) for d in seg_dtypes])
    data, off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    if missing:
        data, off = drop_rows(data, off, set(missing))
    return oseg, data, off


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 63), (3, 64), (4, 65), (5, 255), (6, 256), (7, 257),
                                    (8, 1000), (9, 4099), (10, 20000)])
def test_random_all_dtypes_vs_oracle(ctx, seed, n):
    rng = np.random.default_rng(seed)
    dtypes = list(rng.choice(ALL, size=int(rng.integers(1, 20))))
    dtypes = [D(int(d)) for d in dtypes]
    cols = random_columns(rng, dtypes, n, null_p=float(rng.choice([0.0, 0.1, 0.5, 1.0])))
    missing = set(rng.choice(n, size=n // 10, replace=False).tolist()) if n > 5 else set()
    oseg, data, off = oracle_block(dtypes, cols, n, missing)
    proj = list(rng.integers(0, len(dtypes), size=int(rng.integers(1, 2 * len(dtypes) + 1))))
    seg = seg_of(dtypes)
    got = gpu_decode(ctx, seg, proj, [(data, off)])[0]
    want = O.decode_block(oseg, proj, data, off)
    for p in range(len(proj)):
        assert_array_equal(got[p], want[p], f"seed {seed} proj {p} ({dtypes[proj[p]].name})")
        check_padding(got[p], n)


@pytest.mark.parametrize("max_str,null_p", [(1, 0.0), (3, 0.3), (6, 0.0), (8, 0.1), (8, 0.0), (11, 0.2)])
@pytest.mark.parametrize("n", [1, 7, 64, 129, 3001])
def test_short_strings_packed_stores(ctx, max_str, null_p, n):
    """Short strings (the overlapping head/tail stores of copy_str for 1-8
    bytes; max_str 11 mixes in the 8-byte-step path), nulls and missing rows,
    duplicate projections, several blocks in one launch so chunk edges fall at
    every alignment of the output buffer."""
    rng = np.random.default_rng(1000 * max_str + n)
    dtypes = [D.Utf8, D.Int8, D.Utf8]
    blocks, want = [], []
    for b in range(3):
        cols = random_columns(rng, dtypes, n, null_p=null_p, max_str=max_str, unicode=max_str >= 3)
        missing = set(rng.choice(n, size=n // 7, replace=False).tolist()) if n > 7 else set()
        oseg, data, off = oracle_block(dtypes, cols, n, missing)
        blocks.append((data, off))
        want.append(O.decode_block(oseg, [2, 0, 1, 0], data, off))
    got = gpu_decode(ctx, seg_of(dtypes), [2, 0, 1, 0], blocks)
    for b in range(3):
        for p in range(4):
            assert_array_equal(got[b][p], want[b][p], f"block {b} proj {p}")
            check_padding(got[b][p], n)


def test_long_strings_take_the_hbm_path(ctx):
    # tiles whose blob span exceeds the 32 KiB LDS stage read HBM directly
    rng = np.random.default_rng(11)
    dtypes = [D.Int32, D.Utf8, D.Float64, D.Utf8]
    n = 700
    cols = random_columns(rng, dtypes, n, null_p=0.2, long_every=37, long_len=50000)
    oseg, data, off = oracle_block(dtypes, cols, n, missing={3, 100, 699})
    proj = [1, 0, 3, 2, 1]
    got = gpu_decode(ctx, seg_of(dtypes), proj, [(data, off)])[0]
    want = O.decode_block(oseg, proj, data, off)
    for p in range(len(proj)):
        assert_array_equal(got[p], want[p], f"proj {p}")


def test_multi_block_batch_with_empty_blocks(ctx):
    rng = np.random.default_rng(12)
    dtypes = [D.Float32, D.Utf8, D.Bool, D.UInt64]
    blocks, wants = [], []
    oseg = O.Segment([int(d) for d in dtypes])
    for k, n in enumerate([1000, 0, 257, 1, 0, 3000, 64]):
        cols = random_columns(rng, dtypes, n, null_p=0.1) if n else random_columns(rng, dtypes, 0)
        _, data, off = oracle_block(dtypes, cols, n, missing={0} if n > 2 else set())
        blocks.append((data, off))
        wants.append(O.decode_block(oseg, [1, 0, 2, 3], data, off))
    got = gpu_decode(ctx, seg_of(dtypes), [1, 0, 2, 3], blocks)
    for b in range(len(blocks)):
        for p in range(4):
            assert_array_equal(got[b][p], wants[b][p], f"block {b} proj {p}")


def test_all_rows_missing(ctx):
    dtypes = [D.Utf8, D.Float32]
    n = 300
    data = np.zeros(0, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    got = gpu_decode(ctx, seg_of(dtypes), [0, 1], [(data, off)])[0]
    assert got[0]["null_count"] == n and got[1]["null_count"] == n
    assert np.all(got[0]["offsets"] == 0)
    assert got[1]["values"] == b"\0" * (4 * n)


def test_first_invalid_utf8_error_is_row_major(ctx):
    # ReadBatchBuilder stops at the first failing (row, encoder) pair (read.rs:85-91)
    dtypes = [D.Utf8, D.Utf8]
    n = 2000
    rng = np.random.default_rng(13)
    cols = random_columns(rng, dtypes, n, null_p=0.0, unicode=False)
    oseg, data, off = oracle_block(dtypes, cols, n)
    # corrupt the first non-empty cell at/after row 1500 col 1 and row 1700 col 0
    data = data.copy()
    lens = [np.diff(c["offsets"].astype(np.int64)) for c in cols]
    for r0, c in ((1700, 0), (1500, 1)):
        r = r0 + int(np.argmax(lens[c][r0:] > 0))
        a = int(off[r])
        slot = int.from_bytes(data[a + 1 + 4 * c: a + 5 + 4 * c].tobytes(), "little")
        data[a + 1 + slot + 4] = 0xFF
    with pytest.raises(O.OracleError) as oe:
        O.decode_block(oseg, [0, 1], data, off)
    with pytest.raises(SegmentError, match=r"row %d, column %d" % (oe.value.row, oe.value.column)):
        gpu_decode(ctx, seg_of(dtypes), [0, 1], [(data, off)])


def test_malformed_short_row_reports_instead_of_crashing(ctx):
    dtypes = [D.Float64, D.Utf8]
    data = np.frombuffer(bytes([0xFC, 1, 2, 3]), np.uint8).copy()  # far shorter than bs+cap
    off = np.array([0, 4], np.uint64)
    with pytest.raises(SegmentError, match="malformed"):
        gpu_decode(ctx, seg_of(dtypes), [0], [(data, off)])


def test_zero_projection_is_arrow_error(ctx):
    from murr_amd import ArrowError
    with pytest.raises(ArrowError):
        gpu_decode(ctx, seg_of([D.Float32]), [], [(np.zeros(5, np.uint8), np.array([0, 5], np.uint64))])


@pytest.mark.parametrize("nblocks", [300, 1100])
def test_many_blocks_one_launch(ctx, kernel_mode, nblocks):
    # enough blocks that the JIT kernel's workgroups each own one (300) or
    # several (1100: more blocks than resident workgroups) blocks: the block
    # cursor, per-block null counts, utf8 totals and offsets[0] per block
    rng = np.random.default_rng(13 + nblocks)
    dtypes = [D.Utf8, D.Int64, D.Bool, D.Utf8, D.Float32, D.UInt8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [3, 0, 4, 2, 1, 5, 0]
    blocks, wants = [], []
    for k in range(nblocks):
        n = int(rng.choice([0, 1, 63, 64, 65, 200, 511, 512, 513, 700]))
        cols = random_columns(rng, dtypes, n, null_p=float(rng.choice([0.0, 0.2])), max_str=12)
        miss = set(rng.choice(n, size=n // 7, replace=False).tolist()) if n > 7 else set()
        _, data, off = oracle_block(dtypes, cols, n, miss)
        blocks.append((data, off))
        wants.append(O.decode_block(oseg, proj, data, off))
    got = gpu_decode(ctx, seg_of(dtypes), proj, blocks)
    assert ctx.last_kernel() == KERNEL[kernel_mode]
    for b in range(nblocks):
        for p in range(len(proj)):
            assert_array_equal(got[b][p], wants[b][p], f"block {b} proj {p}")
            check_padding(got[b][p], len(blocks[b][1]) - 1)


@pytest.mark.parametrize("mode,shape,segtiles", [("split", "5x2", 0), ("split", "5x1", 0), ("split", "3x1", 0),
                                                 ("split", "5x3", 0), ("split", "5x2", 1), ("split", "3x1", 2),
                                                 ("local", "5x2", 0), ("local", "3x1", 0), ("local", "5x3", 0)])
def test_split_blocks_utf8_prefix(ctx, kernel_mode, mode, shape, segtiles):
    # few large blocks: in split mode the JIT kernel cuts them into segments
    # (two passes each) and each segment's utf8 starting offsets come from
    # the decoupled look-back over its predecessors; local mode walks every
    # block in one workgroup (forced here to cover it on few blocks)
    nw, r = (int(x) for x in shape.split("x"))
    set_default_opts(kernel=kernel_mode, mode=mode, shape=(nw, r), seg_tiles=segtiles)
    before = ctx.stats()
    rng = np.random.default_rng(40 + len(mode) + int(shape[0]) + segtiles)
    dtypes = [D.Utf8, D.Int16, D.Utf8, D.Bool, D.Float64]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [2, 0, 1, 3, 4, 0]
    blocks, wants = [], []
    for n in [30000, 513, 0, 7777, 1]:
        cols = random_columns(rng, dtypes, n, null_p=0.15, max_str=30)
        miss = set(rng.choice(n, size=n // 9, replace=False).tolist()) if n else set()
        _, data, off = oracle_block(dtypes, cols, n, miss)
        blocks.append((data, off))
        wants.append(O.decode_block(oseg, proj, data, off))
    got = gpu_decode(ctx, seg_of(dtypes), proj, blocks)
    assert ctx.last_kernel() == KERNEL[kernel_mode]
    assert_mode(ctx, before, kernel_mode, mode)
    for b in range(len(blocks)):
        for p in range(len(proj)):
            assert_array_equal(got[b][p], wants[b][p], f"block {b} proj {p}")


def assert_mode(ctx, before, kernel_mode, mode):
    """The decode ran in `mode` (JIT kernel) and no split-mode look-back wait
    expired (an expired wait re-runs the launch in local mode, which would
    hide a broken look-back behind correct output)."""
    st = ctx.stats()
    assert st["split_retries"] == before["split_retries"], "split-mode look-back timed out and was re-run"
    if kernel_mode == "jit":
        assert st["last_mode"] == mode, st


def test_split_many_segments_look_back(ctx, kernel_mode):
    # one block cut into more than 512 one-tile segments: look-backs that span
    # several 512-segment windows and several rounds of the grid
    set_default_opts(kernel=kernel_mode, mode="split", shape=(3, 1), seg_tiles=1)
    before = ctx.stats()
    rng = np.random.default_rng(4242)
    dtypes = [D.Utf8, D.Int32, D.Utf8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [0, 2, 1]
    n = 150000
    cols = random_columns(rng, dtypes, n, null_p=0.1, max_str=12)
    miss = set(rng.choice(n, size=n // 50, replace=False).tolist())
    _, data, off = oracle_block(dtypes, cols, n, miss)
    got = gpu_decode(ctx, seg_of(dtypes), proj, [(data, off)])[0]
    assert_mode(ctx, before, kernel_mode, "split")
    want = O.decode_block(oseg, proj, data, off)
    for p in range(len(proj)):
        assert_array_equal(got[p], want[p], f"proj {p}")


def test_wide_schema_multi_byte_bitset(ctx, kernel_mode):
    # 70 columns (a 9-byte bitset: the per-byte null path) and a 100-column
    # projection with duplicates (more than 64 projected columns)
    rng = np.random.default_rng(77)
    dtypes = [D(int(d)) for d in rng.choice(ALL, size=70)]
    n = 700
    cols = random_columns(rng, dtypes, n, null_p=0.2, max_str=9)
    oseg, data, off = oracle_block(dtypes, cols, n, missing={5, 64, 699})
    proj = [int(x) for x in rng.integers(0, 70, size=100)]
    got = gpu_decode(ctx, seg_of(dtypes), proj, [(data, off)])[0]
    assert ctx.last_kernel() == KERNEL[kernel_mode]
    want = O.decode_block(oseg, proj, data, off)
    for p in range(len(proj)):
        assert_array_equal(got[p], want[p], f"proj {p} ({dtypes[proj[p]].name})")
        check_padding(got[p], n)


@pytest.mark.parametrize("first_null", [0, 63, 511, 512, 4500, 5999])
def test_validity_first_null_late(ctx, kernel_mode, first_null):
    # the JIT kernel writes validity words only once a column has had a null
    # in the block, back-filling the earlier words: place the first null (a
    # null cell, or a missing row) at the start, at tile edges and at the end
    rng = np.random.default_rng(90 + first_null)
    dtypes = [D.Float32, D.Utf8, D.Bool, D.Int64]
    n = 6000
    cols = random_columns(rng, dtypes, n, null_p=0.0, max_str=8)
    for c in cols[:2]:
        v = np.ones(n, bool)
        v[first_null] = False
        v[first_null + 1:] = rng.random(n - first_null - 1) >= 0.3
        c["validity"] = synth.pack_bits(v)
    oseg, data, off = oracle_block(dtypes, cols, n, missing={min(first_null + 7, n - 1)})
    other, odata, ooff = oracle_block(dtypes, random_columns(rng, dtypes, 3000, null_p=0.0), 3000)
    proj = [0, 1, 2, 3, 1]
    got = gpu_decode(ctx, seg_of(dtypes), proj, [(data, off), (odata, ooff)])
    for b, (dd, oo) in enumerate([(data, off), (odata, ooff)]):
        want = O.decode_block(oseg, proj, dd, oo)
        for p in range(len(proj)):
            assert_array_equal(got[b][p], want[p], f"block {b} proj {p}")
            check_padding(got[b][p], len(oo) - 1)


# ---- utf8 index (murr_utf8_index) and the decode of cut blocks ----------------

def utf8_cols(dtypes):
    return [i for i, d in enumerate(dtypes) if d == D.Utf8]


def expected_index(oseg, dtypes, data, off, n, stride):
    """Index entries from the oracle's own decode: column u's utf8 offsets at
    rows 0, stride, 2 stride, ..., and n (the block total)."""
    uc = utf8_cols(dtypes)
    want = O.decode_block(oseg, uc, data, off)
    js = list(range(0, n, stride)) + [n]
    return np.array([[int(want[u]["offsets"][j]) for u in range(len(uc))] for j in js], np.uint64)


@pytest.mark.parametrize("seed,n,stride", [(41, 1, 64), (42, 1000, 64), (43, 4099, 512), (44, 20000, 256),
                                           (45, 70000, 4096)])
def test_utf8_index_matches_oracle_offsets(ctx, seed, n, stride):
    rng = np.random.default_rng(seed)
    dtypes = [D.Utf8, D.Int32, D.Utf8, D.Bool, D.Utf8]
    cols = random_columns(rng, dtypes, n, null_p=0.2, max_str=30)
    oseg, data, off = oracle_block(dtypes, cols, n, set(rng.choice(n, size=n // 9, replace=False).tolist()))
    seg = seg_of(dtypes)
    blk = DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg, stride)
    got = blk.uidx.download().view(np.uint64).reshape(-1, 3)
    assert np.array_equal(got, expected_index(oseg, dtypes, data, off, n, stride))


def test_utf8_index_rows_the_decode_rejects_count_zero(ctx):
    # a malformed cell (slot past the row) and a short row add nothing, as in the decode
    dtypes = [D.Utf8, D.Float32]
    n = 300
    rng = np.random.default_rng(46)
    cols = random_columns(rng, dtypes, n, null_p=0.0, max_str=10)
    oseg, data, off = oracle_block(dtypes, cols, n)
    data = data.copy()
    a = int(off[100])
    data[a + 1: a + 5] = np.frombuffer((10 ** 6).to_bytes(4, "little"), np.uint8)  # slot of row 100
    blk = DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg_of(dtypes), 64)
    got = blk.uidx.download().view(np.uint64)
    lens = np.diff(cols[0]["offsets"].astype(np.int64))
    lens[100] = 0
    want = [int(lens[:j].sum()) for j in list(range(0, n, 64)) + [n]]
    assert got.tolist() == want


@pytest.mark.parametrize("seed,n,nblocks,vrows", [(51, 50000, 1, 0), (52, 30000, 3, 512), (53, 9000, 2, 1024),
                                                  (54, 257, 1, 0)])
def test_cut_blocks_decode_bit_exact(ctx, kernel_mode, seed, n, nblocks, vrows):
    # few large blocks with a utf8 index: local mode over virtual blocks, each
    # starting at its index entry; same buffers as the oracle
    set_default_opts(kernel=kernel_mode, vrows=vrows)
    rng = np.random.default_rng(seed)
    dtypes = [D.Utf8, D.Int64, D.Bool, D.Utf8, D.Float32, D.UInt8, D.Utf8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [3, 0, 4, 2, 1, 5, 6, 0]
    seg = seg_of(dtypes)
    dblocks, wants = [], []
    for b in range(nblocks):
        cols = random_columns(rng, dtypes, n, null_p=0.15, max_str=20)
        _, data, off = oracle_block(dtypes, cols, n, set(rng.choice(n, size=n // 11, replace=False).tolist()))
        dblocks.append(DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg, 512))
        wants.append(O.decode_block(oseg, proj, data, off))
    outs = decode_blocks(ctx, seg, proj, dblocks)
    for b, blk in enumerate(dblocks):
        for p, ci in enumerate(proj):
            got = download_array(ctx, outs.array(b, p), int(seg.columns[ci].dtype), n)
            assert_array_equal(got, wants[b][p], f"block {b} proj {p}")
            check_padding(got, n)


def test_cut_blocks_first_error_is_row_major(ctx, kernel_mode):
    dtypes = [D.Utf8, D.Utf8]
    n = 40000
    rng = np.random.default_rng(55)
    cols = random_columns(rng, dtypes, n, null_p=0.0, unicode=False)
    oseg, data, off = oracle_block(dtypes, cols, n)
    data = data.copy()
    lens = [np.diff(c["offsets"].astype(np.int64)) for c in cols]
    for r0, c in ((31000, 0), (23000, 1)):
        r = r0 + int(np.argmax(lens[c][r0:] > 0))
        a = int(off[r])
        slot = int.from_bytes(data[a + 1 + 4 * c: a + 5 + 4 * c].tobytes(), "little")
        data[a + 1 + slot + 4] = 0xFF
    with pytest.raises(O.OracleError) as oe:
        O.decode_block(oseg, [0, 1], data, off)
    seg = seg_of(dtypes)
    blk = DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg, 256)
    with pytest.raises(SegmentError, match=r"row %d, column %d" % (oe.value.row, oe.value.column)):
        decode_blocks(ctx, seg, [0, 1], [blk])


def test_layout_without_utf8_cuts_without_index(ctx, kernel_mode):
    dtypes = [D.Int64, D.Float32, D.Bool, D.UInt16]
    n = 60000
    rng = np.random.default_rng(56)
    cols = random_columns(rng, dtypes, n, null_p=0.3)
    oseg, data, off = oracle_block(dtypes, cols, n, {5, 6, 59999})
    seg = seg_of(dtypes)
    blk = DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg, 512)
    assert blk.uidx is None  # nothing to index
    proj = [3, 2, 1, 0]
    outs = decode_blocks(ctx, seg, proj, [blk])
    want = O.decode_block(oseg, proj, data, off)
    for p, ci in enumerate(proj):
        assert_array_equal(download_array(ctx, outs.array(0, p), int(seg.columns[ci].dtype), n), want[p], f"proj {p}")


@pytest.mark.parametrize("shape", ["5x3", "5x2", "3x1"])
def test_validity_local_whole_blocks(ctx, kernel_mode, shape):
    # local mode over whole blocks, several per workgroup: a column's first
    # null at tile edges, in the last row, as a missing row, in one column but
    # not the others, or none at all; every buffer bit-exact when null_count >
    # 0 (round 5 measured storing validity lazily from a block's first null
    # on -- slower on config B; this pins the cases it needed)
    nw, r = (int(x) for x in shape.split("x"))
    set_default_opts(kernel=kernel_mode, mode="local", shape=(nw, r))
    rng = np.random.default_rng(300 + nw * 10 + r)
    dtypes = [D.Utf8, D.Float32, D.Bool, D.Int16, D.Utf8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [0, 1, 2, 3, 4, 1]
    n = 6000
    blocks, wants = [], []
    cases = [(None, None), (0, None), (63, None), (64, None), (767, None), (768, 1), (1535, 3),
             (5000, None), (n - 1, None), ("missing", 2000), (None, 4500)]
    for first, other in cases:
        cols = random_columns(rng, dtypes, n, null_p=0.0, max_str=9)
        miss = set()
        if first == "missing":
            miss = {other}  # a missing row: null in every column
        else:
            if first is not None:  # column 0's first null
                v = np.ones(n, bool)
                v[first] = False
                v[first + 1:] = rng.random(n - first - 1) >= 0.2
                cols[0]["validity"] = synth.pack_bits(v)
            if other is not None:  # column 3 (int16) nulls from row `other` on
                v = np.ones(n, bool)
                v[other:] = rng.random(n - other) >= 0.5
                v[other] = False
                cols[3]["validity"] = synth.pack_bits(v)
        _, data, off = oracle_block(dtypes, cols, n, miss)
        blocks.append((data, off))
        wants.append(O.decode_block(oseg, proj, data, off))
    got = gpu_decode(ctx, seg_of(dtypes), proj, blocks * 3)  # 33 blocks: several per workgroup
    for b in range(len(blocks) * 3):
        for p in range(len(proj)):
            assert_array_equal(got[b][p], wants[b % len(blocks)][p], f"block {b} proj {p}")
            check_padding(got[b][p], n)


PAIR_DTYPES = [D.Int8, D.UInt16, D.Bool, D.UInt8, D.Int16, D.Int8, D.Bool, D.Utf8, D.Int64, D.UInt16]


@pytest.mark.parametrize("proj", [list(range(10)), [0, 1, 2], [3, 4, 6], [4, 3, 1, 0, 9, 5], [5, 9, 2, 6],
                                  [0, 3, 0, 3, 1, 4, 7]], ids=["all", "firsts", "seconds", "rev", "odd", "dup"])
@pytest.mark.parametrize("mode,shape", [("local", "5x3"), ("local", "5x2"), ("local", "3x1"), ("split", "3x1"),
                                        ("split", "5x2")])
def test_narrow_pairs_and_bool_words(ctx, kernel_mode, mode, shape, proj):
    # narrow (1- and 2-byte) columns in pairs and alone, and bool columns,
    # whose value words the JIT kernel writes in the validity store's lanes
    # (word lane NCOLS + c); projections holding both, one or neither of a
    # pair (round 5 measured pairing two narrow columns into one store: no
    # faster), ragged chunk ends, nulls and missing rows; every
    # buffer bit-exact against the oracle
    nw, r = (int(x) for x in shape.split("x"))
    set_default_opts(kernel=kernel_mode, mode=mode, shape=(nw, r))
    rng = np.random.default_rng(500 + nw * 10 + r + len(mode) + len(proj))
    oseg = O.Segment([int(d) for d in PAIR_DTYPES])
    blocks, wants = [], []
    for n in [9000, 1, 63, 65, 200, 4097]:
        cols = random_columns(rng, PAIR_DTYPES, n, null_p=0.2, max_str=12)
        miss = set(rng.choice(n, size=n // 13, replace=False).tolist()) if n > 13 else set()
        _, data, off = oracle_block(PAIR_DTYPES, cols, n, miss)
        blocks.append((data, off))
        wants.append((n, O.decode_block(oseg, proj, data, off)))
    got = gpu_decode(ctx, seg_of(PAIR_DTYPES), proj, blocks * 2)
    for b in range(len(blocks) * 2):
        n, want = wants[b % len(blocks)]
        for p in range(len(proj)):
            assert_array_equal(got[b][p], want[p], f"block {b} proj {p}")
            check_padding(got[b][p], n)
