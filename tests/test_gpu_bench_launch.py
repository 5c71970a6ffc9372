"""bench.py's headline launch, checked block by block: 1000 resident config-B
blocks of 100k FLOAT32+UTF8 rows, written by the device encoder with their
utf8 index (stride 512), decoded by one prepared plan (murr_decode_plan /
murr_decode_run) in the default shape and mode -- exactly the launch
bench.py times.  Unlike the bench, the blocks here are not all copies of one:
eight distinct sources rotate over the 1000 slots, so a block decoded into
another block's outputs (or from another block's bytes) shows up.  The first,
the last, two random blocks and one block of every source are compared with
the oracle's decode after repeated runs; the launch must not have needed the
split-abort retry."""
import os
import sys

import numpy as np
import pytest

import oracle as O
from murr_amd import synth
from murr_amd.device import Context, DecodeOutputs, DecodePlan, encode_block, set_default_opts
from murr_amd.schema import SegmentSchema

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu
ROWS, K, SOURCES, STRIDE = 100_000, 1000, 8, 512


def test_bench_config_b_launch_block_by_block():
    set_default_opts()  # bench's default shape and mode
    ctx = Context(0)
    plan = None
    try:
        srcs, hosts = [], []
        for s in range(SOURCES):
            cols = bench.make_columns("B", ROWS, start=s * ROWS)
            seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
            b = encode_block(ctx, seg, synth.upload_columns(ctx, cols), ROWS, STRIDE)
            srcs.append(b)
            hosts.append((b.data.download(b.data_bytes),
                          b.row_off.download(8 * (ROWS + 1)).view(np.uint64).copy()))
        blocks = [srcs[i] if i < SOURCES else bench.copy_block(ctx, srcs[i % SOURCES]) for i in range(K)]
        proj = [0, 1]
        outs = DecodeOutputs(ctx, seg, proj, blocks)
        plan = DecodePlan(ctx, seg, proj, blocks, outs)
        before = ctx.stats()["split_retries"]
        for _ in range(4):
            plan.run()
        st = ctx.stats()
        assert st["split_retries"] == before, st
        assert ctx.last_kernel() == "murr_jit_decode"

        rng = np.random.default_rng(2024)
        check = {0, K - 1, *rng.choice(np.arange(1, K - 1), 2, replace=False).tolist(), *range(SOURCES)}
        oseg = O.Segment([int(c.dtype) for c in seg.columns])
        want = [O.decode_block(oseg, proj, *h) for h in hosts]
        for b in sorted(check):
            s = b % SOURCES
            bad, _ = bench.verify_arrays(ctx, seg, proj, outs, b, *hosts[s], want=want[s])
            assert not bad, bad
    finally:
        if plan is not None:
            plan.close()
        ctx.close()
