"""Blocks with u32 row offsets (murr_block_t.row_off32, round 5): the same
decode, bit for bit, as their u64 form and as the oracle -- on both kernels,
in every work mode (local, split, cut on a utf8 index), at any 4-byte
alignment of the offsets, and mixed with u64 blocks in one launch.  The
reference stores a row's bytes whole (src/io/row/write.rs:19-52) and reads them
back in caller order (src/io/row/read.rs:85-98); the offsets' width is this
library's own layout of a batch and changes no output byte."""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal
from randgen import ALL, drop_rows, random_columns
from murr_amd import SegmentError, synth
from murr_amd.device import Context, DeviceBlock, DeviceBuffer, decode_blocks, download_array, set_default_opts
from murr_amd.errors import MurrError
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    set_default_opts(kernel=request.param)
    yield request.param
    set_default_opts()


def seg_of(dtypes):
    return SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])


def oracle_block(dtypes, cols, n, missing=()):
    oseg = O.Segment([int(d) for d in dtypes])
    data, off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    if missing:
        data, off = drop_rows(data, off, set(missing))
    return oseg, data, off


class _Slice(DeviceBuffer):
    """A window into another device buffer (the parent owns the memory)."""

    def __init__(self, parent, offset, nbytes):
        self.ctx, self.ptr, self.nbytes, self._parent = parent.ctx, parent.ptr + offset, nbytes, parent

    def free(self):
        self.ptr = 0


def block32(ctx, data, off, lead=0):
    """A u32 block whose offsets start `lead` dwords past a 16-B boundary."""
    o32 = np.zeros(lead + off.size, np.uint32)
    o32[lead:] = off.astype(np.uint32)
    buf = ctx.upload(o32)
    return DeviceBlock(ctx.upload(data), None, off.size - 1, int(data.size),
                       row_off32=_Slice(buf, 4 * lead, 4 * off.size))


def decode_check(ctx, seg, proj, dblocks, wants):
    outs = decode_blocks(ctx, seg, proj, dblocks)
    for b, blk in enumerate(dblocks):
        for p, ci in enumerate(proj):
            got = download_array(ctx, outs.array(b, p), int(seg.columns[ci].dtype), blk.n_rows)
            assert_array_equal(got, wants[b][p], f"block {b} proj {p}")


@pytest.mark.parametrize("seed,n,lead", [(1, 1, 0), (2, 63, 1), (3, 64, 2), (4, 65, 3), (5, 257, 0),
                                         (6, 1000, 1), (7, 4099, 2), (8, 20000, 3), (9, 100000, 0)])
def test_random_all_dtypes_u32_vs_oracle(ctx, seed, n, lead):
    rng = np.random.default_rng(500 + seed)
    dtypes = [D(int(d)) for d in rng.choice(ALL, size=int(rng.integers(1, 18)))]
    cols = random_columns(rng, dtypes, n, null_p=float(rng.choice([0.0, 0.1, 0.5])))
    missing = set(rng.choice(n, size=n // 10, replace=False).tolist()) if n > 5 else set()
    oseg, data, off = oracle_block(dtypes, cols, n, missing)
    proj = [int(x) for x in rng.integers(0, len(dtypes), size=int(rng.integers(1, 2 * len(dtypes) + 1)))]
    decode_check(ctx, seg_of(dtypes), proj, [block32(ctx, data, off, lead)], [O.decode_block(oseg, proj, data, off)])


@pytest.mark.parametrize("nblocks", [40, 1100])
def test_mixed_widths_one_launch(ctx, nblocks):
    # u32 and u64 blocks side by side (the block cursor switches width per
    # block), several blocks per workgroup at 1100; every lead
    rng = np.random.default_rng(77 + nblocks)
    dtypes = [D.Utf8, D.Int64, D.Bool, D.Utf8, D.Float32, D.UInt8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [3, 0, 4, 2, 1, 5, 0]
    seg = seg_of(dtypes)
    dblocks, wants = [], []
    for k in range(nblocks):
        n = int(rng.choice([0, 1, 63, 64, 65, 200, 511, 700, 1300]))
        cols = random_columns(rng, dtypes, n, null_p=float(rng.choice([0.0, 0.2])), max_str=12)
        miss = set(rng.choice(n, size=n // 7, replace=False).tolist()) if n > 7 else set()
        _, data, off = oracle_block(dtypes, cols, n, miss)
        dblocks.append(block32(ctx, data, off, k % 4) if k % 3 else DeviceBlock.upload(ctx, data, off))
        wants.append(O.decode_block(oseg, proj, data, off))
    decode_check(ctx, seg, proj, dblocks, wants)


@pytest.mark.parametrize("mode,shape,segtiles", [("split", "5x2", 0), ("split", "3x1", 1), ("split", "5x3", 0),
                                                 ("local", "5x3", 0), ("local", "3x1", 0)])
def test_split_and_local_u32(ctx, kernel_mode, mode, shape, segtiles):
    nw, r = (int(x) for x in shape.split("x"))
    set_default_opts(kernel=kernel_mode, mode=mode, shape=(nw, r), seg_tiles=segtiles)
    before = ctx.stats()
    rng = np.random.default_rng(90 + nw + r + segtiles)
    dtypes = [D.Utf8, D.Int16, D.Utf8, D.Bool, D.Float64]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [2, 0, 1, 3, 4, 0]
    dblocks, wants = [], []
    for i, n in enumerate([30000, 513, 0, 7777, 1]):
        cols = random_columns(rng, dtypes, n, null_p=0.15, max_str=30)
        miss = set(rng.choice(n, size=n // 9, replace=False).tolist()) if n else set()
        _, data, off = oracle_block(dtypes, cols, n, miss)
        dblocks.append(block32(ctx, data, off, i % 4))
        wants.append(O.decode_block(oseg, proj, data, off))
    decode_check(ctx, seg_of(dtypes), proj, dblocks, wants)
    st = ctx.stats()
    assert st["split_retries"] == before["split_retries"]
    if kernel_mode == "jit":
        assert st["last_mode"] == mode, st


@pytest.mark.parametrize("seed,n,nblocks,stride,lead", [(61, 50000, 1, 512, 0), (62, 30000, 3, 128, 1),
                                                        (63, 9000, 2, 256, 3)])
def test_cut_u32_blocks_on_their_index(ctx, kernel_mode, seed, n, nblocks, stride, lead):
    # the utf8 index built from the u32 offsets equals the u64 one, and the
    # cut decode over it is bit-exact
    rng = np.random.default_rng(seed)
    dtypes = [D.Utf8, D.Int64, D.Bool, D.Utf8, D.Float32, D.UInt8, D.Utf8]
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [3, 0, 4, 2, 1, 5, 6, 0]
    seg = seg_of(dtypes)
    dblocks, wants = [], []
    for b in range(nblocks):
        cols = random_columns(rng, dtypes, n, null_p=0.15, max_str=20)
        _, data, off = oracle_block(dtypes, cols, n, set(rng.choice(n, size=n // 11, replace=False).tolist()))
        b32 = block32(ctx, data, off, lead).index_utf8(ctx, seg, stride)
        b64 = DeviceBlock.upload(ctx, data, off).index_utf8(ctx, seg, stride)
        assert np.array_equal(b32.uidx.download(), b64.uidx.download())
        dblocks.append(b32)
        wants.append(O.decode_block(oseg, proj, data, off))
    decode_check(ctx, seg, proj, dblocks, wants)


def test_u32_first_error_is_row_major(ctx, kernel_mode):
    dtypes = [D.Utf8, D.Utf8]
    n = 40000
    rng = np.random.default_rng(65)
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
    for blk in (block32(ctx, data, off, 2), block32(ctx, data, off, 0).index_utf8(ctx, seg, 256)):
        with pytest.raises(SegmentError, match=r"row %d, column %d" % (oe.value.row, oe.value.column)):
            decode_blocks(ctx, seg, [0, 1], [blk])


def test_narrow_equals_host_cast_and_refuses_overflow(ctx, kernel_mode):
    rng = np.random.default_rng(66)
    off = np.concatenate([[0], np.cumsum(rng.integers(0, 90, size=70001))]).astype(np.uint64)
    b64 = DeviceBlock(ctx.alloc(16), ctx.upload(off), off.size - 1, int(off[-1]))
    b32 = b64.narrow(ctx)
    assert b32.row_off is None and b32.offset_width == 4
    assert np.array_equal(b32.row_off32.download().view(np.uint32), off.astype(np.uint32))
    big = off.copy()
    big[-1] = 1 << 32
    with pytest.raises(MurrError, match="overflow"):
        DeviceBlock(ctx.alloc(16), ctx.upload(big), big.size - 1, 0).narrow(ctx)
    # every offset is checked, not only the last: an interior one
    # past 2^32 in a malformed block is not truncated into a plausible span
    mid = off.copy()
    mid[35000] += 1 << 32
    with pytest.raises(MurrError, match="overflow"):
        DeviceBlock(ctx.alloc(16), ctx.upload(mid), mid.size - 1, 0).narrow(ctx)
    dec = off.copy()
    dec[50000] = dec[49999] - 1 if dec[49999] else 0
    dec[49999] += 5
    with pytest.raises(SegmentError, match="malformed"):
        DeviceBlock(ctx.alloc(16), ctx.upload(dec), dec.size - 1, 0).narrow(ctx)


def test_config_b_block_u32_matches_u64(ctx, kernel_mode):
    # the headline's block (configs[1]: 100k rows of f32 + utf8) through the
    # device encode, narrowed on the device: both widths give the oracle's
    # buffers
    from murr_amd.device import encode_block
    n = 100_000
    cols = synth.config_b(n)
    seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
    b64 = encode_block(ctx, seg, synth.upload_columns(ctx, cols), n, 512)
    b32 = b64.narrow(ctx)
    data = b64.data.download(b64.data_bytes)
    off = b64.row_off.download(8 * (n + 1)).view(np.uint64)
    assert np.array_equal(b32.host_offsets(), off)
    oseg = O.Segment([int(c["dtype"]) for c in cols])
    want = O.decode_block(oseg, [0, 1], data, off)
    decode_check(ctx, seg, [0, 1], [b32, b64], [want, want])
