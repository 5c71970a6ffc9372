"""Decode error paths the reference panics on, reported instead: the utf8 i32
offset overflow (arrow-rs StringBuilder panics past i32::MAX,
src/io/codec/utf8.rs:86-96) and an output buffer too small for the strings
(MURR_E_CAPACITY with the exact bytes required).  The first error is the
reference's: row-major, then projection order (ReadBatchBuilder::add_row,
src/io/row/read.rs:85-91).  Both kernels."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from randgen import random_columns
from murr_amd import _abi, synth
from murr_amd.device import Context, DecodeOutputs, DeviceBlock, set_default_opts
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu
MIB = 1 << 20


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


def big_block(n, lens):
    """n rows of len(lens) non-null utf8 columns, column c's strings all
    lens[c] bytes of 'a' (WriteRow layout, src/io/row/write.rs:19-52)."""
    nc = len(lens)
    cap = 4 * nc
    row = 1 + cap + sum(4 + L for L in lens)
    data = np.full(n * row + 16, 0x61, np.uint8)
    rows = data[: n * row].reshape(n, row)
    rows[:, 0] = 0xFF & ~((1 << nc) - 1)
    slot = cap
    for c, L in enumerate(lens):
        rows[:, 1 + 4 * c: 5 + 4 * c] = np.frombuffer(int(slot).to_bytes(4, "little"), np.uint8)
        rows[:, 1 + slot: 5 + slot] = np.frombuffer(int(L).to_bytes(4, "little"), np.uint8)
        slot += 4 + L
    off = np.arange(n + 1, dtype=np.uint64) * row
    return data, off


def decode_status(ctx, seg, proj, blocks, outs=None):
    outs = outs or DecodeOutputs(ctx, seg, proj, blocks)
    cb = (_abi.Block * len(blocks))()
    for i, b in enumerate(blocks):
        cb[i].data, cb[i].row_off, cb[i].n_rows, cb[i].data_bytes = b.data.ptr, b.row_off.ptr, b.n_rows, b.data_bytes
    pj = (C.c_uint32 * len(proj))(*proj)
    err = _abi.Error()
    st = ctx.L.murr_decode_blocks(ctx.h, C.byref(seg.c), pj, len(proj), cb, len(blocks), outs.arrays, C.byref(err))
    return st, err, outs


@pytest.fixture(scope="module")
def overflow_block(ctx):
    # column 1's strings pass i32::MAX at row 511 (512 x 4 MiB = 2^31 bytes)
    data, off = big_block(520, [1, 4 * MIB])
    blk = DeviceBlock.upload(ctx, data, off)
    del data
    return blk


@pytest.mark.parametrize("proj,col", [([1], 0), ([0, 1], 1), ([1, 0], 0), ([0, 0, 1], 2)])
def test_offset_overflow_first_row_row_major(ctx, overflow_block, proj, col):
    seg = SegmentSchema([("s", D.Utf8), ("big", D.Utf8)])
    st, err, _ = decode_status(ctx, seg, proj, [overflow_block])
    assert st == _abi.E_OFFSET_OVERFLOW, _abi.status_str(st)
    assert (err.block, err.row, err.column) == (0, 511, col)


def test_small_column_of_the_overflow_block_decodes(ctx, overflow_block):
    # the other column's offsets stay far below i32::MAX: no error
    seg = SegmentSchema([("s", D.Utf8), ("big", D.Utf8)])
    st, err, outs = decode_status(ctx, seg, [0], [overflow_block])
    assert st == _abi.OK
    assert outs.array(0, 0).data_len == 520


def small_outs(ctx, seg, proj, blocks, caps):
    """DecodeOutputs whose utf8 values buffers hold caps[(block, proj)] bytes."""
    outs = DecodeOutputs(ctx, seg, proj, blocks)
    for (b, p), cap in caps.items():
        a = outs.array(b, p)
        buf = ctx.alloc(max(cap, 8))
        outs.bufs.append(buf)
        a.values, a.values_cap = buf.ptr, cap
    return outs


@pytest.mark.parametrize("nblocks", [1, 3])
def test_capacity_reports_exact_required(ctx, nblocks):
    rng = np.random.default_rng(17 + nblocks)
    dtypes = [D.Int32, D.Utf8, D.Utf8]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    oseg = O.Segment([int(d) for d in dtypes])
    blocks, hosts = [], []
    for b in range(nblocks):
        cols = random_columns(rng, dtypes, 5000, null_p=0.1, max_str=30)
        data, off = O.encode_batch(oseg, synth.oracle_cols(cols), 5000)
        blocks.append(DeviceBlock.upload(ctx, data, off))
        hosts.append((data, off))
    proj = [0, 2, 1]
    bad = nblocks - 1  # the undersized buffer: last block, projection position 1 (column 2)
    want = O.decode_block(oseg, proj, *hosts[bad])
    offs = want[1]["offsets"].astype(np.int64)
    total = int(offs[-1])
    cap = total // 3
    st, err, outs = decode_status(ctx, seg, proj, blocks, small_outs(ctx, seg, proj, blocks, {(bad, 1): cap}))
    assert st == _abi.E_CAPACITY, _abi.status_str(st)
    first = int(np.argmax(offs[1:] > cap))  # first row whose string ends past the buffer
    assert (err.block, err.row, err.column) == (bad, first, 1)
    assert err.required == total
