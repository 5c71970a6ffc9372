"""Per-workgroup timeline of one config-D shard decode (tuning library built
with `make tuning`, MURR_JIT_DEFS=MJ_TIMELINE=1, MURR_DECODE_VERBOSE=1): the
non-plan decode path prints start / first-tile / end percentiles."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from murr_amd.device import Context, decode_blocks, parse_opts, set_default_opts  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
if os.environ.get("UIDX_STRIDE"):  # experiment: the table's utf8 index stride
    import murr_amd.resident
    murr_amd.resident.UIDX_STRIDE = int(os.environ["UIDX_STRIDE"])
if len(sys.argv) > 2:
    set_default_opts(**parse_opts(sys.argv[2]))
ctx = Context(0)
rt, names = bench.config_d_table(ctx, rows, 0)
blk = rt.block()
proj = list(range(len(rt.segment.columns)))
for i in range(3):
    t = time.perf_counter()
    decode_blocks(ctx, rt.segment, proj, [blk])
    print(f"run {i}: kernel {ctx.last_kernel_ms():.4f} ms, call {1e3 * (time.perf_counter() - t):.3f} ms", file=sys.stderr)
ctx.close()
