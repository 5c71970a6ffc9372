"""bench.py's headline launch, checked block by block: 1000 resident config-B
blocks of 100k FLOAT32+UTF8 rows, written by the device encoder with their
utf8 index (stride 512), decoded by one prepared plan (murr_decode_plan /
murr_decode_run) in the default shape and mode -- exactly the launch
bench.py times.  Unlike the bench, the blocks here are not all copies of one:
eight distinct sources rotate over the 1000 slots, so a block decoded into
another block's outputs (or from another block's bytes) shows up.  The first,
the last, two random blocks and one block of every source are compared with
the oracle's decode after repeated runs; the launch must not have needed the
split-abort retry.  Both offset widths: u32 (row_off32, the bench's default
since round 5) and u64.  Then bench.py itself, whose line must be
self-consistent: the kernel time it reports never exceeds its step."""
import json
import os
import subprocess
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


@pytest.mark.parametrize("width", [32, 64])
def test_bench_config_b_launch_block_by_block(width):
    set_default_opts()  # bench's default shape and mode
    ctx = Context(0)
    plan = None
    try:
        srcs, hosts = [], []
        for s in range(SOURCES):
            cols = bench.make_columns("B", ROWS, start=s * ROWS)
            seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
            b = encode_block(ctx, seg, synth.upload_columns(ctx, cols), ROWS, STRIDE)
            if width == 32:
                b = b.narrow(ctx, keep64=True)
            hosts.append((b.data.download(b.data_bytes),
                          b.row_off.download(8 * (ROWS + 1)).view(np.uint64).copy()))
            if width == 32:
                assert np.array_equal(b.host_offsets(), hosts[-1][1])
                b.row_off = None  # the decode sees the u32 offsets only
            srcs.append(b)
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


def test_bench_line_is_self_consistent():
    """bench.py's own line (a shorter run of the headline launch): verified
    against the oracle, u32 offsets counted at 4 B per row, and kernel_ms_avg
    (GPU marks around the timed region / steps) <= ms_per_step (the host
    clock around the same steps)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "12", "--warmup", "3",
                          "--blocks", "300", "--no-cpu", "--no-traffic"],
                         capture_output=True, text=True, timeout=240, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    rf = line["roofline"]
    assert line["verified"].startswith("blocks"), line["verified"]
    assert line["config"]["row_offset_bytes"] == 4
    assert rf["kernel_ms_avg"] <= line["ms_per_step"], (rf["kernel_ms_avg"], line["ms_per_step"])
    assert rf["frac_step"] <= rf["frac"] + 1e-9
    assert line["config"]["bytes_in_per_step"] == 300 * (1788890 + 4 * 100001 + 1576)
    _lane_policy(line)


def _lane_policy(line):
    # one rule for every config -- the line is per launch (one
    # stream), the overlapped rate is the extra `lanes` key with every lane's
    # last output verified
    assert line["lane_policy"].startswith("per launch"), line["lane_policy"]
    ln = line["lanes"]
    assert ln["lanes"] == 3 and ln["verified"].startswith("every lane"), ln
    assert ln["frac_step_lanes"] > 0 and ln["ms_per_step"] > 0


def test_bench_line_config_d_same_lane_policy():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", "D", "--rows", "300000",
                          "--steps", "9", "--warmup", "3", "--no-cpu", "--no-traffic"],
                         capture_output=True, text=True, timeout=240, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["verified"].startswith("blocks"), line["verified"]
    assert line["roofline"]["kernel_ms_avg"] <= line["ms_per_step"]
    _lane_policy(line)
