"""Prepared decodes (murr_decode_plan / murr_decode_run): a run gives the
same buffers and counts as murr_decode_blocks_ix on the same inputs, picks
up changed block bytes (same addresses and sizes) on the next run, and covers
every launch form: whole blocks, blocks cut on their utf8 index, split mode,
duplicate projections (several rounds), empty blocks, both kernels."""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal
from randgen import random_columns
from murr_amd import SegmentError, _abi, synth
from murr_amd.device import Context, DecodeOutputs, DecodePlan, DeviceBlock, download_array, set_default_opts
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


def make(rng, dtypes, n, nulls=0.1):
    cols = random_columns(rng, dtypes, n, null_p=nulls, max_str=14) if n else random_columns(rng, dtypes, 0)
    oseg = O.Segment([int(d) for d in dtypes])
    data, off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
    return oseg, data, off


def check(ctx, seg, oseg, proj, hosts, outs, tag):
    for b, (data, off) in enumerate(hosts):
        n = off.size - 1
        want = O.decode_block(oseg, proj, data, off)
        for p, ci in enumerate(proj):
            got = download_array(ctx, outs.array(b, p), int(seg.columns[ci].dtype), n)
            assert_array_equal(got, want[p], f"{tag} block {b} proj {p}")


@pytest.mark.parametrize("form", ["whole", "cut", "split", "dup"])
def test_plan_runs_match_the_oracle(ctx, kernel_mode, form):
    rng = np.random.default_rng(hash(form) % 1000)
    dtypes = [D.Utf8, D.Float32, D.Bool, D.Utf8, D.Int64]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    sizes = {"whole": [700, 0, 300, 64, 1], "cut": [40000, 9000], "split": [30000, 513], "dup": [2000, 0, 77]}[form]
    proj = [3, 0, 1, 2, 4, 0] if form == "dup" else [4, 3, 2, 1, 0]
    hosts, blocks = [], []
    for n in sizes:
        oseg, data, off = make(rng, dtypes, n)
        hosts.append((data, off))
        blk = DeviceBlock.upload(ctx, data, off)
        if form == "cut":
            blk.index_utf8(ctx, seg, 512)
        blocks.append(blk)
    if form in ("split", "whole"):
        ctx.set_opts(kernel=kernel_mode, mode="split" if form == "split" else "local")
    try:
        plan = DecodePlan(ctx, seg, proj, blocks)
        for rnd in range(2):
            plan.run()
            check(ctx, seg, oseg, proj, hosts, plan.outs, f"{form} run {rnd}")
        st = ctx.stats()
        assert st["split_retries"] == 0 and st["readback_fallbacks"] == 0, st
        if kernel_mode == "jit":
            assert st["last_mode"] == {"whole": "local", "cut": "cut", "split": "split", "dup": "split"}[form], st
        plan.close()
    finally:
        ctx.set_opts(kernel=kernel_mode)


def test_plan_rereads_changed_bytes(ctx, kernel_mode):
    # same sizes, new contents: the next run decodes the new bytes
    rng = np.random.default_rng(3)
    dtypes = [D.Int32, D.Utf8]
    seg = SegmentSchema([("a", D.Int32), ("b", D.Utf8)])
    oseg, d1, off = make(rng, dtypes, 5000, nulls=0.0)
    blk = DeviceBlock.upload(ctx, d1, off)
    plan = DecodePlan(ctx, seg, [1, 0], [blk])
    plan.run()
    check(ctx, seg, oseg, [1, 0], [(d1, off)], plan.outs, "first")
    d2 = d1.copy()
    # flip int32 payload bytes of every row (the row layout, hence the sizes, is unchanged)
    starts = off[:-1].astype(np.int64)
    d2[starts + 1] ^= 0x5A
    blk.data.copy_from(DeviceBlock.upload(ctx, d2, off).data, d2.size)
    plan.run()
    check(ctx, seg, oseg, [1, 0], [(d2, off)], plan.outs, "second")
    plan.close()


def test_plan_reports_errors_each_run(ctx, kernel_mode):
    dtypes = [D.Utf8]
    seg = SegmentSchema([("s", D.Utf8)])
    rng = np.random.default_rng(4)
    oseg, data, off = make(rng, dtypes, 3000, nulls=0.0)
    data = data.copy()
    r = int(np.argmax(np.diff(off.astype(np.int64)) > 5))
    a = int(off[r])
    data[a + 1 + int.from_bytes(data[a + 1:a + 5].tobytes(), "little") + 4] = 0xFF
    blk = DeviceBlock.upload(ctx, data, off)
    plan = DecodePlan(ctx, seg, [0], [blk])
    for _ in range(2):
        with pytest.raises(SegmentError, match=f"row {r},"):
            plan.run()
    plan.close()


def test_two_plans_alternating_async_runs(ctx, kernel_mode):
    # murr_decode_run_async / _wait with two plans (two output sets) on one
    # context, the next run launched before the previous is waited for, as
    # bench.py times the headline: every run's buffers and counts as the oracle
    rng = np.random.default_rng(71)
    dtypes = [D.Float32, D.Utf8, D.Int16]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    proj = [0, 1, 2]
    hosts, blocks = [], []
    for n in [5000, 70000, 0, 1300]:
        oseg, data, off = make(rng, dtypes, n)
        hosts.append((data, off))
        blocks.append(DeviceBlock.upload(ctx, data, off))
    plans = [DecodePlan(ctx, seg, proj, blocks) for _ in range(2)]
    plans[0].run_async()
    for s in range(5):
        if s + 1 < 5:
            plans[(s + 1) % 2].run_async()
        outs = plans[s % 2].wait()
        assert ctx.last_kernel_ms() >= 0.0
        check(ctx, seg, oseg, proj, hosts, outs, f"run {s}")
    # sampled timing: the plan's timed runs (one in PLAN_TIME_EVERY) report
    # a kernel time, the others leave the last timed run's in place
    # (plans[0] has run 3 times: its next runs are numbered 3, 4, ...)
    e = _abi.PLAN_TIME_EVERY
    ks = []
    for r in range(3, 3 + 2 * e + 1):
        plans[0].run()
        ks.append((r, ctx.last_kernel_ms()))
    assert all(k > 0.0 for _, k in ks)
    last = {}
    for r, k in ks:
        last.setdefault(r - r % e, []).append(k)
    for t, group in last.items():  # (the generic kernel's plans time every run)
        if kernel_mode != "generic":
            assert len(set(group)) == 1, (t, group)  # untimed runs repeat the timed run's time
    with pytest.raises(Exception):
        plans[0].wait()  # nothing in flight
    plans[0].run_async()
    with pytest.raises(Exception):
        plans[0].run_async()  # one run of a plan in flight at a time
    plans[0].wait()
    for p in plans:
        p.close()


def test_split_plans_overlapped_on_three_streams(kernel_mode):
    # Three split-mode launches of more segments than one grid round, on three
    # contexts (streams) at once, so they compete for the CUs.  Segments are
    # claimed in the order workgroups run (murr_jit_kernel.hip seg_claim):
    # with the static deal a resident workgroup's look-back waited on a
    # workgroup of its own launch that other launches kept off the GPU, every
    # wait ran to its bound and the launch was re-run in local mode
    # (split_retries; bench.py's C no-index lanes took 21 ms a step).
    if kernel_mode != "jit":
        pytest.skip("split mode is the JIT kernel's")
    rng = np.random.default_rng(606)
    dtypes = [D.Utf8, D.Int32, D.Utf8]
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    oseg, data, off = make(rng, dtypes, 400000)
    proj = [0, 2, 1]
    ctxs = [Context(0) for _ in range(3)]
    try:
        plans = []
        for c in ctxs:
            c.set_opts(kernel="jit", mode="split", shape=(3, 1), seg_tiles=1)  # 3125 one-tile segments
            plans.append(DecodePlan(c, seg, proj, [DeviceBlock.upload(c, data, off)]))
        for _ in range(3):
            for p in plans:
                p.run_async()
            for p in plans:
                p.wait()
        for c, p in zip(ctxs, plans):
            st = c.stats()
            assert st["split_retries"] == 0 and st["last_mode"] == "split", st
            check(c, seg, oseg, proj, [(data, off)], p.outs, "overlapped split")
            p.close()
    finally:
        for c in ctxs:
            c.close()
