"""Streaming host decode (murr_hstream_*): batch reads back to back, host
memory in and out, pipelined over several slots -- every returned batch
bit-exact against the oracle's ReadBatchBuilder restatement
(src/io/row/read.rs:62-110), from pinned and from pageable sources, with
missing rows, empty and one-row batches, blocks that start mid-buffer, and a
malformed batch that fails alone (ReadBatchBuilder::build's error) while the
batches around it decode.  Row offsets as u64 (murr_hstream_submit) and as
u32 (murr_hstream_submit32)."""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal
from randgen import ALL, drop_rows, random_columns
from murr_amd import synth
from murr_amd.device import Context, encode_batch
from murr_amd.errors import MurrError, SegmentError
from murr_amd.row import HostBuffer, HostStream, host_array_buffers
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def encode_host(ctx, seg, cols, n):
    blob, off, blen = encode_batch(ctx, seg, synth.upload_columns(ctx, cols), n)
    return blob.download(blen).copy(), off.download(8 * (n + 1)).view(np.uint64).copy()


def check(outs, oseg, proj, data, off, what):
    want = O.decode_block(oseg, proj, data, off)
    for p in range(len(proj)):
        assert_array_equal(host_array_buffers(outs[p]), want[p], f"{what} col {p}")


@pytest.mark.parametrize("depth,pinned,width", [(2, False, 64), (3, True, 64), (4, False, 64), (8, True, 64),
                                                (2, False, 32), (3, True, 32), (8, True, 32)])
def test_stream_random_batches_vs_oracle(ctx, depth, pinned, width):
    rng = np.random.default_rng(100 + depth)
    dtypes = [D.Utf8, D.Int32, D.Bool, D.Float64, D.Utf8, D.UInt8, D.Int16, D.Int64, D.UInt64, D.Float32,
              D.Int8, D.UInt16, D.UInt32]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    oseg = O.Segment([int(d) for d in dtypes])
    proj = [4, 0, 2, 1, 3, 12, 0]
    sizes = [1000, 0, 1, 4099, 257, 20000, 64, 3000, 9, 1500]
    batches = []
    for k, n in enumerate(sizes):
        cols = random_columns(rng, dtypes, n, null_p=0.15, max_str=30)
        data, off = encode_host(ctx, seg, cols, n) if n else (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        if n > 10:
            data, off = drop_rows(data, off, set(rng.integers(0, n, size=n // 10).tolist()))
        batches.append((data, off))
    hs = HostStream(seg, proj, depth=depth, ctx=ctx)
    keep = []
    odt = np.uint32 if width == 32 else np.uint64

    def submit(k):
        data, off = batches[k]
        off = off.astype(odt)
        if pinned:
            hb, ho = HostBuffer(data.size + 16, ctx), HostBuffer(off.nbytes, ctx)
            hb.array[: data.size] = data
            ho.array[:] = off.view(np.uint8)
            keep.append((hb, ho))
            hs.submit(hb.array, ho.array.view(odt), pinned=True)
        else:
            # a scratch copy the caller overwrites right after submit: the
            # library staged it already
            d2, o2 = data.copy(), off.copy()
            hs.submit(d2, o2)
            d2[:] = 0xAB
            o2[:] = 0

    nxt = 0
    while nxt < depth and nxt < len(sizes):
        submit(nxt)
        nxt += 1
    with pytest.raises(MurrError):
        submit(nxt)  # every slot holds a batch not yet returned
    for k in range(len(sizes)):
        outs = hs.next()
        check(outs, oseg, proj, *batches[k], f"batch {k} (n={sizes[k]})")
        if nxt < len(sizes):
            submit(nxt)
            nxt += 1
    st = hs.stats()
    assert st["batches"] == len(sizes) and st["h2d_bytes"] > 0 and st["d2h_bytes"] > 0
    with pytest.raises(MurrError):
        hs.next()  # nothing left to return
    hs.close()


@pytest.mark.parametrize("width,pinned", [(64, True), (32, True), (32, False)])
def test_stream_config_b_full_size_every_block(ctx, width, pinned):
    # configs[1]'s 100k-row FLOAT32 + UTF8 blocks, 12 batches through three
    # slots from a ring of four: every block bit-exact.  Pageable sources
    # above 1 MiB are staged by the copy pool's threads, batch after batch
    # (each copy's pieces are its own job: no worker of an earlier copy can
    # touch the next one's)
    n, ring = 100_000, 4
    odt = np.uint32 if width == 32 else np.uint64
    seg = SegmentSchema([("f", D.Float32), ("s", D.Utf8)])
    oseg = O.Segment([int(D.Float32), int(D.Utf8)])
    srcs = []
    for r in range(ring):
        cols = synth.config_b(n, start=r * n, null_frac=0.05 if r % 2 else 0.0, seed=r)
        data, off = encode_host(ctx, seg, cols, n)
        o = off.astype(odt)
        hb, ho = HostBuffer(data.size + 16, ctx), HostBuffer(o.nbytes, ctx)
        hb.array[: data.size] = data
        ho.array[:] = o.view(np.uint8)
        srcs.append((hb, ho, data, off))
    hs = HostStream(seg, [0, 1], depth=3, ctx=ctx)
    total, nxt = 12, 0

    def submit(i):
        hb, ho, data, off = srcs[i % ring]
        if pinned:
            hs.submit(hb.array, ho.array.view(odt), pinned=True)
        else:
            hs.submit(data, off.astype(odt))

    while nxt < 3:
        submit(nxt)
        nxt += 1
    for k in range(total):
        outs = hs.next()
        _, _, data, off = srcs[k % ring]
        check(outs, oseg, [0, 1], data, off, f"batch {k}")
        if nxt < total:
            submit(nxt)
            nxt += 1
    hs.close()


def test_stream_block_starting_mid_buffer(ctx):
    # row offsets that do not start at 0 (a slice of a larger cache page):
    # only the block's own bytes travel, the decode sees the same rows
    rng = np.random.default_rng(7)
    dtypes = [D.Utf8, D.Float32]
    seg = SegmentSchema([("s", D.Utf8), ("f", D.Float32)])
    oseg = O.Segment([int(d) for d in dtypes])
    cols = random_columns(rng, dtypes, 5000, null_p=0.1)
    data, off = encode_host(ctx, seg, cols, 5000)
    hs = HostStream(seg, [0, 1], depth=2, ctx=ctx)
    off32 = off.astype(np.uint32)
    for lo, hi, w in [(37, 4000, 64), (1, 2, 64), (4999, 5000, 64), (0, 5000, 64), (37, 4000, 32), (3, 5000, 32)]:
        sub = off[lo:hi + 1] if w == 64 else off32[lo:hi + 1]  # (u32: offsets at any 4-byte alignment)
        hs.submit(data, sub)
        outs = hs.next()
        base = int(off[lo])
        check(outs, oseg, [0, 1], data[base:int(off[hi])].copy(), (sub - off[lo]).astype(np.uint64),
              f"rows {lo}..{hi}")
    hs.close()


def test_stream_malformed_batch_fails_alone(ctx):
    rng = np.random.default_rng(3)
    dtypes = [D.Utf8, D.Int64]
    seg = SegmentSchema([("s", D.Utf8), ("i", D.Int64)])
    oseg = O.Segment([int(d) for d in dtypes])
    good = [encode_host(ctx, seg, random_columns(rng, dtypes, 700, null_p=0.2), 700) for _ in range(3)]
    bad_data, bad_off = good[1][0].copy(), good[1][1].copy()
    # row 5 cut to 3 bytes: shorter than its fixed part (read.rs:39-55 bounds)
    row5 = bad_data[int(bad_off[5]):int(bad_off[5]) + 3].tobytes()
    parts = [bad_data[: int(bad_off[5])].tobytes(), row5, bad_data[int(bad_off[6]):].tobytes()]
    shift = int(bad_off[6] - bad_off[5]) - 3
    bad_off[6:] -= shift
    bad_data = np.frombuffer(b"".join(parts), np.uint8).copy()
    hs = HostStream(seg, [0, 1], depth=3, ctx=ctx)
    hs.submit(*good[0])
    hs.submit(bad_data, bad_off)
    hs.submit(*good[2])
    check(hs.next(), oseg, [0, 1], *good[0], "before")
    with pytest.raises(SegmentError, match=r"row 5,"):  # MURR_E_MALFORMED_ROW at row 5
        hs.next()
    check(hs.next(), oseg, [0, 1], *good[2], "after")
    hs.close()


def test_stream_pinned_buffer_rewritten_between_batches(ctx):
    # one pinned source buffer refilled with a different batch each time (the
    # copy reads it over PCIe at its device address: no stale bytes from the
    # batch before), and batches of every size through the same slots
    rng = np.random.default_rng(11)
    dtypes = [D.Utf8, D.Int64, D.Bool, D.Utf8]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    oseg = O.Segment([int(d) for d in dtypes])
    batches = [encode_host(ctx, seg, random_columns(rng, dtypes, n, null_p=0.2, max_str=40), n)
               for n in (3000, 17, 3000, 2500, 1)]
    cap = max(d.size for d, _ in batches) + 16
    hb, ho = HostBuffer(cap, ctx), HostBuffer(8 * 3001, ctx)
    hs = HostStream(seg, [3, 0, 1, 2], depth=2, ctx=ctx)
    for k, (data, off) in enumerate(batches):
        hb.array[:] = 0x5A
        hb.array[: data.size] = data
        ho.array[: off.nbytes] = off.view(np.uint8)
        hs.submit(hb.array, ho.array.view(np.uint64)[: off.size], pinned=True)
        check(hs.next(), oseg, [3, 0, 1, 2], data, off, f"batch {k}")
    hs.close()
