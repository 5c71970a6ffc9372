"""The utf8 index as a product artifact, and whole-table scans.

* murr_encode_batch_ix writes a block's index with the block; its entries are
  the oracle decode's own utf8 offsets at every stride.
* ResidentTable.write keeps the arena's index as it grows (appends of odd
  sizes: only the new rows are indexed, murr_utf8_index_update), and so does
  load_sst.
* ResidentTable.scan decodes the whole arena in one launch cut on that index
  (config D's "each GPU decodes its whole shard"), bit-exact against the
  oracle's decode of the same blob -- at 1.25 M config-C rows too.
"""
import ctypes as C

import numpy as np
import pyarrow as pa
import pytest

import oracle as O
from golden_util import assert_array_equal
from randgen import random_columns
from murr_amd import synth
from murr_amd.device import Context, DecodeOutputs, download_array, encode_block, set_default_opts
from murr_amd.resident import UIDX_STRIDE, ResidentTable
from murr_amd.schema import DTypeName as D, SegmentSchema

from test_gpu_resident import C_DTYPES, batch_c, schema_c

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def index_of(oseg, dtypes, data, off, n, stride):
    uc = [i for i, d in enumerate(dtypes) if d == D.Utf8]
    want = O.decode_block(oseg, uc, data, off)
    js = list(range(0, n, stride)) + [n]
    return np.array([[int(want[u]["offsets"][j]) for u in range(len(uc))] for j in js], np.uint64)


@pytest.mark.parametrize("n,stride", [(1, 64), (1000, 64), (4099, 512), (30000, 256)])
def test_encode_block_writes_the_index(ctx, n, stride):
    rng = np.random.default_rng(n)
    dtypes = [D.Utf8, D.Int16, D.Utf8, D.Bool]
    cols = random_columns(rng, dtypes, n, null_p=0.2, max_str=20)
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    blk = encode_block(ctx, seg, synth.upload_columns(ctx, cols), n, stride)
    oseg = O.Segment([int(d) for d in dtypes])
    data, off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    assert blk.data.download(blk.data_bytes).tobytes() == data.tobytes()
    got = blk.uidx.download().view(np.uint64).reshape(-1, 2)
    assert np.array_equal(got, index_of(oseg, dtypes, data, off, n, stride))


def test_encode_block_without_utf8_has_no_index(ctx):
    seg = SegmentSchema([("a", D.Float32), ("b", D.Int64)])
    cols = synth.config_e(100, ncols=1) + [synth.column(D.Int64, np.arange(100))]
    blk = encode_block(ctx, seg, synth.upload_columns(ctx, cols), 100)
    assert blk.uidx is None and blk.n_rows == 100


def arena(rt):
    data = rt.arena.download(rt.used)
    off = rt.row_off.download(8 * (rt.n + 1)).view(np.uint64).copy()
    return data, off


@pytest.mark.parametrize("kernel", ["jit", "generic"])
def test_resident_appends_keep_the_index_and_scan(ctx, kernel):
    set_default_opts(kernel=kernel)
    try:
        rt = ResidentTable(schema_c(), ctx)
        sizes = [1000, 777, 1, 513, 4099, 512, 3]
        start = 0
        for k, m in enumerate(sizes):
            rt.write(batch_c(m, start=start, seed=40 + k))
            start += m
            data, off = arena(rt)
            oseg = O.Segment([int(d) for d in C_DTYPES])
            want_ix = index_of(oseg, C_DTYPES, data, off, rt.n, UIDX_STRIDE)
            got_ix = rt.uidx.download(8 * want_ix.size).view(np.uint64).reshape(want_ix.shape)
            assert np.array_equal(got_ix, want_ix), f"after append {k}"
        names = [f"c{i}" for i in range(len(C_DTYPES))]
        proj = [12, 0, 11, 3, 12]
        outs = rt.scan_device([names[i] for i in proj])
        st = ctx.stats()
        if kernel == "jit":
            assert st["last_mode"] == "cut", st
        want = O.decode_block(oseg, proj, data, off)
        for p, ci in enumerate(proj):
            assert_array_equal(download_array(ctx, outs.array(0, p), int(C_DTYPES[ci]), rt.n), want[p], f"proj {p}")
        # the host form: the written rows in write order
        whole = pa.Table.from_batches([batch_c(m, start=sum(sizes[:k]), seed=40 + k)
                                       for k, m in enumerate(sizes)]).combine_chunks()
        got = rt.scan(["c12", "c0", "c4"])
        for name, col in zip(["c12", "c0", "c4"], got.columns):
            assert col.equals(whole.column(name).combine_chunks()), name
    finally:
        set_default_opts()


def test_scan_device_bit_exact_config_d_shard(ctx):
    # config D's per-GPU work: one 1.25 M-row shard of the config-C schema,
    # decoded whole in one launch over the arena cut on its index
    n = 1_250_000
    rt = ResidentTable(schema_c(), ctx)
    rt.write(batch_c(n))
    names = [f"c{i}" for i in range(len(C_DTYPES))]
    outs = rt.scan_device(names)
    assert ctx.last_kernel() == "murr_jit_decode"
    st = ctx.stats()
    assert st["last_mode"] == "cut" and st["split_retries"] == 0, st
    data, off = arena(rt)
    oseg = O.Segment([int(d) for d in C_DTYPES])
    want = O.decode_block(oseg, list(range(len(C_DTYPES))), data, off)
    for p, d in enumerate(C_DTYPES):
        assert_array_equal(download_array(ctx, outs.array(0, p), int(d), n), want[p], f"col {p}")
    # the outputs are reused across scans of the same shard
    again = rt.scan_device(names, outs)
    assert again is outs
    for p in (0, 11, 12):
        assert_array_equal(download_array(ctx, outs.array(0, p), int(C_DTYPES[p]), n), want[p], f"again {p}")


def test_scan_device_async_alternating_outputs(ctx):
    # two output sets, the next scan launched before the previous is waited
    # for (bench.py's timed loop for config D): each keeps its own prepared
    # plan and both hold the oracle's arrays
    n = 200_000
    rt = ResidentTable(schema_c(), ctx)
    rt.write(batch_c(n))
    names = [f"c{i}" for i in range(len(C_DTYPES))]
    first = rt.scan_device(names)
    sets = [DecodeOutputs(ctx, rt.segment, list(range(len(C_DTYPES))), [rt.block()]) for _ in range(2)]
    h = rt.scan_device_async(names, sets[0])
    for s in range(4):
        hn = rt.scan_device_async(names, sets[(s + 1) % 2]) if s < 3 else None
        assert h.wait() is sets[s % 2]
        h = hn
    data, off = arena(rt)
    want = O.decode_block(O.Segment([int(d) for d in C_DTYPES]), list(range(len(C_DTYPES))), data, off)
    for outs in sets + [first]:
        for p in (0, 3, 11, 12, 15):
            assert_array_equal(download_array(ctx, outs.array(0, p), int(C_DTYPES[p]), n), want[p], f"col {p}")


def test_scan_plan_eviction_with_runs_in_flight(ctx):
    # five output sets scanned without waiting: the plan cache holds four, so
    # one plan is evicted while its run is in flight.  Eviction finishes that
    # run first; every handle's wait() still returns its own, correct outputs
    # (a freed plan under a running launch)
    n = 20_000
    rt = ResidentTable(schema_c(), ctx)
    rt.write(batch_c(n, seed=7))
    names = [f"c{i}" for i in range(len(C_DTYPES))]
    sets = [DecodeOutputs(ctx, rt.segment, list(range(len(C_DTYPES))), [rt.block()]) for _ in range(5)]
    hs = [rt.scan_device_async(names, s) for s in sets]
    data, off = arena(rt)
    want = O.decode_block(O.Segment([int(d) for d in C_DTYPES]), list(range(len(C_DTYPES))), data, off)
    for h, outs in zip(hs, sets):
        assert h.wait() is outs
        for p in (0, 11, 12):
            assert_array_equal(download_array(ctx, outs.array(0, p), int(C_DTYPES[p]), n), want[p], f"col {p}")
    with pytest.raises(ValueError):
        hs[0].wait()  # its one result was handed over already


@pytest.mark.parametrize("nlanes", [2, 3])
def test_scan_device_lanes_overlap(ctx, nlanes):
    # bench.py --config D's default loop (--lanes 3): one output set per
    # lane, each on its own context of one device (its own stream), nlanes - 1
    # scans launched ahead of the one waited for, so they overlap on the GPU.
    # Every scan of every lane reads the same arena; each output set holds
    # the oracle's arrays after its last scan
    n = 300_000
    rt = ResidentTable(schema_c(), ctx)
    rt.write(batch_c(n, seed=11))
    names = [f"c{i}" for i in range(len(C_DTYPES))]
    extra = [Context(ctx.device) for _ in range(nlanes - 1)]
    try:
        lanes = [ctx] + extra
        sets = [DecodeOutputs(c, rt.segment, list(range(len(C_DTYPES))), [rt.block()]) for c in lanes]
        steps = 3 * nlanes
        inflight = [rt.scan_device_async(names, sets[s], ctx=lanes[s]) for s in range(nlanes - 1)]
        for s in range(steps):
            if s + nlanes - 1 < steps:
                k = (s + nlanes - 1) % nlanes
                inflight.append(rt.scan_device_async(names, sets[k], ctx=lanes[k]))
            assert inflight.pop(0).wait() is sets[s % nlanes]
        data, off = arena(rt)
        want = O.decode_block(O.Segment([int(d) for d in C_DTYPES]), list(range(len(C_DTYPES))), data, off)
        for k, outs in enumerate(sets):
            for p, d in enumerate(C_DTYPES):
                assert_array_equal(download_array(ctx, outs.array(0, p), int(d), n), want[p], f"lane {k} col {p}")
    finally:
        for _, plan in rt._scan_plans.values():  # (plans on the extra lanes close before they do)
            plan.close()
        rt._scan_plans.clear()
        for c in extra:
            c.close()
