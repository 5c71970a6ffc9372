"""Per-workgroup timeline of one config-B launch (1000 x 100k-row blocks), or
with TIMELINE_CONFIG=C of config C's (10 x 1M-row blocks, utf8 index 512;
tuning library built with `make tuning`, MURR_JIT_DEFS=MJ_TIMELINE=1,
MURR_DECODE_VERBOSE=1): the non-plan decode path prints start / first-tile /
end percentiles and the last end per XCD (MURR_TIMELINE_DUMP: per workgroup)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from murr_amd import synth  # noqa: E402
from murr_amd.device import Context, decode_blocks, encode_block, parse_opts, set_default_opts  # noqa: E402
from murr_amd.schema import SegmentSchema  # noqa: E402

config = os.environ.get("TIMELINE_CONFIG", "B")
blocks_n = int(sys.argv[1]) if len(sys.argv) > 1 else (1000 if config == "B" else 10)
if len(sys.argv) > 2:
    set_default_opts(**parse_opts(sys.argv[2]))
ctx = Context(0)
rows = 100_000 if config == "B" else 1_000_000
cols = bench.make_columns(config, rows, start=0)
seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
dcols = synth.upload_columns(ctx, cols)
b0 = encode_block(ctx, seg, dcols, rows, 512)
blocks = [b0] + [bench.copy_block(ctx, b0) for _ in range(blocks_n - 1)]
ctx.sync()
for i in range(3):
    t = time.perf_counter()
    decode_blocks(ctx, seg, list(range(len(cols))), blocks)
    print(f"run {i}: kernel {ctx.last_kernel_ms():.4f} ms, call {1e3 * (time.perf_counter() - t):.3f} ms", file=sys.stderr)
ctx.close()
