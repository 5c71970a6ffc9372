#!/usr/bin/env python3
"""Block-decode throughput of murr's row-blob codec on MI355X.

Metric (BASELINE.json): block-decode GiB/s, device-resident, Arrow bytes out,
at 1/2/4/8 GPUs.  One step = one murr_decode_blocks call (one kernel launch)
over K blocks of configs[1]'s shape ("read_block shape: 100k-row
FLOAT32+UTF8"), inputs already resident in HBM; the step includes the
readback of null counts / string lengths the caller needs to assemble the
Arrow arrays.  Multi-GPU (torchrun, one process per GPU): every rank decodes its
own key-range shard (weak scaling), no data-path collective; torch.distributed
(gloo, CPU) carries only the barrier and the max-over-ranks timing.

Extra modes (not the headline line): --mode host (pinned H2D + decode + D2H
through the batched ReadBatchBuilder), --mode encode (configs[4] write shape),
--config C/D (16-col mixed nullable).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import murr_amd  # noqa: E402  (the HIP library is loaded in main(), after the rank spawn decision)
from murr_amd import _abi, synth  # noqa: E402
from murr_amd.device import Context, DecodeOutputs, DecodePlan, DeviceBlock, DeviceBuffer, device_count, encode_batch, \
    encode_block, parse_opts, set_default_opts  # noqa: E402
from murr_amd.schema import DTypeName as D, SegmentSchema  # noqa: E402
from murr_amd.shard import Group, shard_rows  # noqa: E402


METRIC = "block-decode GiB/s device-resident (Arrow bytes out) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); no MFMA on this path
GIB = float(1 << 30)


def dist_init(args):
    g = Group("gloo")
    return g, g.rank, g.world, g.local_rank


def barrier(g):
    g.barrier()


def max_over_ranks(g, x: float) -> float:
    return g.max(x)


def sum_over_ranks(g, x: float) -> float:
    return g.sum(x)


def make_columns(config: str, rows: int, start: int):
    if config == "A":
        return synth.config_a(rows, start=start)
    if config == "B":
        return synth.config_b(rows, start=start)
    if config in ("C", "D"):
        return synth.config_c(rows, start=start)
    if config == "E":
        return synth.config_e(rows, start=start)
    raise SystemExit(f"unknown config {config}")


def parse_proj(text, ncols):
    """--proj: comma-separated columns, "rev" (every column, reversed), or
    None (every column in order: the whole-table projection)."""
    if text is None:
        return list(range(ncols))
    if text == "rev":
        return list(reversed(range(ncols)))
    return [int(x) for x in text.split(",")]


def arrow_out_bytes(seg, proj, n, null_counts, utf8_lens):
    """SURVEY.md §8(d) bytes_out: values + offsets + string bytes + validity of
    columns that have nulls."""
    tot = 0
    for p, ci in enumerate(proj):
        d = int(seg.columns[ci].dtype)
        if d == 0:
            tot += 4 * (n + 1) + utf8_lens[p]
        elif d == 1:
            tot += (n + 7) // 8
        else:
            tot += n * _abi.lib().murr_dtype_size(d)
        if null_counts[p]:
            tot += (n + 7) // 8
    return tot


def pmc_traffic(paths, kernel=None):
    """HBM bytes per decode launch from rocprofv3 --pmc CSVs (comma-separated;
    FETCH_SIZE and WRITE_SIZE come from separate passes).  MI355X_MICROARCH.md
    §HBM: FETCH_SIZE counts half the bytes of wide streaming reads on gfx950,
    so it is doubled; WRITE_SIZE is exact for 16-B stores; both in KiB.
    kernel: only dispatches of that kernel (the timed launch's; the untimed
    no-index variant runs another one)."""
    if not paths:
        return None
    import csv
    fetch, write = [], []
    for path in paths.split(","):
        if not os.path.exists(path):
            return None
        per = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if "decode" not in name or (kernel and name.split("(")[0].strip() != kernel):
                    continue
                key = (r.get("Counter_Name"), r.get("Dispatch_Id"))
                per[key] = per.get(key, 0.0) + float(r.get("Counter_Value", 0))
        for (name, _), v in per.items():
            (fetch if name == "FETCH_SIZE" else write if name == "WRITE_SIZE" else []).append(v)
    if not fetch or not write:
        return None
    return round((2.0 * sum(fetch) / len(fetch) + sum(write) / len(write)) * 1024.0)


def measure_traffic(args, kernel):
    """roofline.traffic of this very configuration, measured: the bench
    re-runs itself (2 steps) under `rocprofv3 --pmc FETCH_SIZE`, then under
    `--pmc WRITE_SIZE` (one counter per pass, never with a trace domain), as
    child processes after the timed region, and pmc_traffic reads the
    timed kernel's dispatches.  None when rocprofv3 is absent or a pass fails
    (each pass is bounded to 150 s and killed with its process group)."""
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    # never nested: a bench already running under rocprofv3 (its tool library
    # preloaded, ROCPROF_* set) leaves the counters to that profiler
    if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ):
        return None
    keep = [a for a in sys.argv[1:]]
    drop = {"--steps", "--warmup", "--gpus"}
    argv, skip = [], False
    for a in keep:
        if skip:
            skip = False
            continue
        if a in drop:
            skip = True
            continue
        if a.split("=")[0] in drop or a in ("--no-cpu", "--no-traffic"):
            continue
        argv.append(a)
    paths = []
    with tempfile.TemporaryDirectory(prefix="murr_pmc_") as d:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            # the interpreter's resolved path after `--` (a `python3` looked up
            # on PATH may be a wrapper that execs the real one, and rocprofv3
            # itself execs what follows `--`)
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", ctr.lower(), "--",
                   os.path.realpath(sys.executable), os.path.abspath(__file__), *argv, "--steps", "2", "--warmup", "1",
                   "--no-cpu", "--no-traffic"]
            env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
            pr = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env,
                                  start_new_session=True)
            try:
                rc = pr.wait(timeout=150)
            except subprocess.TimeoutExpired:
                os.killpg(pr.pid, signal.SIGKILL)
                pr.wait()
                return None
            path = os.path.join(d, f"{ctr.lower()}_counter_collection.csv")
            if rc != 0 or not os.path.exists(path):
                return None
            paths.append(path)
        return pmc_traffic(",".join(paths), kernel)


def cpu_model() -> str:
    """The host CPU's model name (lscpu model next to every
    CPU number), from /proc/cpuinfo."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.lower().startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(seg, proj, host_blob, host_off, rows, target_s):
    """The oracle (C restatement of ReadBatchBuilder, 1 thread) on this host."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    oseg = O.Segment([int(c.dtype) for c in seg.columns])
    t = time.perf_counter()
    res = O.decode_block(oseg, proj, host_blob, host_off)
    one = time.perf_counter() - t
    out_bytes = arrow_out_bytes(seg, proj, rows, [r["null_count"] for r in res],
                                [len(r["values"]) if r["dtype"] == 0 else 0 for r in res])
    reps = int(max(1, min(100000, target_s / max(one, 1e-6))))
    t = time.perf_counter()
    for _ in range(reps):
        O.decode_block(oseg, proj, host_blob, host_off)
    dt = time.perf_counter() - t
    return {"value": round(out_bytes * reps / dt / GIB, 4), "unit": "GiB/s", "cores": 1,
            "kind": "port", "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{reps} blocks x {rows} rows of the same workload decoded by "
                      f"oracle/libmurr_oracle.so (serial ReadBatchBuilder restatement), {dt:.1f} s"}


def host_cores():
    """Host threads this process may really use, and where the number comes
    from (all cores, stated): the CPU affinity mask, capped by
    the cgroup's CPU quota (v2 cpu.max or v1 cfs_quota_us / cfs_period_us;
    the GPU box's share is a quota over a 256-thread host).  Counts hardware
    threads: two per physical core on an SMT host (`smt` in the source)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota, qsrc = None, None
    for path, kind in (("/sys/fs/cgroup/cpu.max", "v2"), ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "v1")):
        try:
            with open(path) as f:
                txt = f.read().split()
            if kind == "v2":
                if txt and txt[0] != "max":
                    quota, qsrc = int(txt[0]) / int(txt[1]), "cgroup v2 cpu.max"
            else:
                q = int(txt[0])
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    per = int(f.read().split()[0])
                if q > 0:
                    quota, qsrc = q / per, "cgroup v1 cfs_quota_us"
            break
        except (OSError, ValueError, IndexError):
            continue
    smt = 1
    try:
        with open("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list") as f:
            sib = f.read().strip()
        smt = sum(int(b) - int(a) + 1 if "-" in r else 1
                  for r in sib.split(",") for a, _, b in [r.partition("-")])
    except (OSError, ValueError):
        pass
    n = aff
    src = f"sched_getaffinity {aff}"
    if quota is not None:
        n = max(1, min(aff, int(quota)))
        src += f", {qsrc} {quota:g} CPUs"
    return n, f"{src} -> {n} threads ({smt} hardware thread(s) per core)"


def cpu_baseline_threads(seg, proj, host_blob, host_off, rows, target_s, threads):
    """Upper bound the reference does not implement: the
    same oracle on `threads` host threads, each decoding a contiguous row range
    of the block (ctypes drops the GIL inside the C call)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    oseg = O.Segment([int(c.dtype) for c in seg.columns])
    parts = []
    for t in range(threads):
        r0, r1 = rows * t // threads, rows * (t + 1) // threads
        b0, b1 = int(host_off[r0]), int(host_off[r1])
        parts.append((host_blob[b0:b1].copy(), (host_off[r0:r1 + 1] - host_off[r0]).astype(np.uint64), r1 - r0))
    part_bytes = []
    for blob, off, n in parts:
        res = O.decode_block(oseg, proj, blob, off)
        part_bytes.append(arrow_out_bytes(seg, proj, n, [r["null_count"] for r in res],
                                          [len(r["values"]) if r["dtype"] == 0 else 0 for r in res]))
    done = [0] * threads
    deadline = time.perf_counter() + target_s

    def work(i):
        blob, off, _ = parts[i]
        while time.perf_counter() < deadline:
            O.decode_block(oseg, proj, blob, off)
            done[i] += 1
    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t
    total = sum(d * b for d, b in zip(done, part_bytes))
    return {"value": round(total / dt / GIB, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"{sum(done)} row-range parts ({threads} per block of {rows} rows) on {threads} "
                      f"threads, oracle/libmurr_oracle.so, {dt:.1f} s"}


def L_len(ctx, seg, rows, stride):
    return ctx.L.murr_utf8_index_len(C.byref(seg.c), rows, stride)


def check_gpus(local_rank, world):
    ndev = device_count()
    if local_rank >= ndev:
        # one GPU per rank: more ranks than GPUs would share a GPU and report a
        # wrong aggregate, so refuse instead of wrapping around
        raise SystemExit(f"local rank {local_rank} has no GPU of its own: {ndev} visible, WORLD_SIZE {world}")


class _View(DeviceBuffer):
    """A piece of an arena buffer (the arena owns the memory)."""

    def __init__(self, parent: DeviceBuffer, offset: int, nbytes: int):
        self.ctx, self.ptr, self.nbytes, self._parent = parent.ctx, parent.ptr + offset, nbytes, parent

    def free(self):
        self.ptr = 0


class _Arena:
    """Pieces of one device buffer, each at a multiple of `align` bytes."""

    def __init__(self, ctx, sizes, align: int):
        self.offs, off = [], 0
        for n in sizes:
            self.offs.append(off)
            off += (n + align - 1) // align * align
        self.buf = ctx.alloc(max(off, 16))
        self.sizes = list(sizes)

    def view(self, i: int) -> _View:
        return _View(self.buf, self.offs[i], self.sizes[i])


def arena_blocks(ctx, b0: DeviceBlock, K: int, align: int):
    """K resident copies of a block in three arenas (blobs, row offsets,
    utf8 indexes), each piece at a multiple of `align` bytes (--arena)."""
    w = b0.offset_width
    src_off = b0.row_off32 if w == 4 else b0.row_off
    nd, no = b0.data_bytes + 16, w * (b0.n_rows + 1)
    ad, ao = _Arena(ctx, [nd] * K, align), _Arena(ctx, [no] * K, align)
    au = _Arena(ctx, [b0.uidx.nbytes] * K, 256) if b0.uidx is not None else None
    out = []
    for i in range(K):
        d, o = ad.view(i), ao.view(i)
        d.copy_from(b0.data, b0.data_bytes)
        o.copy_from(src_off, no)
        u = None
        if au is not None:
            u = au.view(i)
            u.copy_from(b0.uidx, b0.uidx.nbytes)
        out.append(DeviceBlock(d, None if w == 4 else o, b0.n_rows, b0.data_bytes, u, b0.stride,
                               o if w == 4 else None))
    return out


class ArenaOutputs(DecodeOutputs):
    """DecodeOutputs with every buffer a piece of one arena (--arena)."""

    def __init__(self, ctx, segment, proj, blocks, align: int):
        self.ctx, self.proj, self.blocks = ctx, list(proj), blocks
        np_ = len(self.proj)
        self.arrays = (_abi.Array * max(len(blocks) * np_, 1))()
        L = ctx.L
        plan = []  # (array index, field, bytes)
        for b, blk in enumerate(blocks):
            n = blk.n_rows
            bm = int(L.murr_bitmap_bytes(n))
            for p, ci in enumerate(self.proj):
                col = segment.columns[ci]
                i = b * np_ + p
                if col.dtype == D.Utf8:
                    vb = max(blk.data_bytes, 8)
                    plan.append((i, "offsets", (n + 1) * 4))
                    self.arrays[i].values_cap = vb
                elif col.dtype == D.Bool:
                    vb = bm
                else:
                    vb = n * col.dtype.size()
                plan += [(i, "values", max(vb, 8)), (i, "validity", max(bm, 8))]
        self.arena = _Arena(ctx, [x[2] for x in plan], align)
        self.bufs = [self.arena.buf]
        for k, (i, field, _) in enumerate(plan):
            setattr(self.arrays[i], field, self.arena.view(k).ptr)


def copy_block(ctx, b: DeviceBlock) -> DeviceBlock:
    """A resident copy of a block (its offsets at their width, and its
    index), device to device."""
    w = b.offset_width
    data, off = ctx.alloc(b.data_bytes + 16), ctx.alloc(w * (b.n_rows + 1))
    data.copy_from(b.data, b.data_bytes)
    off.copy_from(b.row_off32 if w == 4 else b.row_off, w * (b.n_rows + 1))
    ux = None
    if b.uidx is not None:
        ux = ctx.alloc(b.uidx.nbytes)
        ux.copy_from(b.uidx, b.uidx.nbytes)
    return DeviceBlock(data, None if w == 4 else off, b.n_rows, b.data_bytes, ux, b.stride,
                       off if w == 4 else None)


def config_d_table(ctx, rows: int, start: int, chunk: int = 2_000_000, stride: int = 0):
    """Config D's shard: the config-C schema with keys "key{i}", rows
    [start, start + rows), written into a ResidentTable (device encode, key
    index, utf8 index kept by every write)."""
    import pyarrow as pa
    from murr_amd import ColumnSchema, TableSchema
    from murr_amd.resident import ResidentTable
    cols_s = {"key": ColumnSchema(D.Utf8, False)}
    cols_s.update({f"c{i}": ColumnSchema(c["dtype"]) for i, c in enumerate(synth.config_c(1))})
    from murr_amd.resident import UIDX_STRIDE
    rt = ResidentTable(TableSchema("key", cols_s), ctx, uidx_stride=stride or UIDX_STRIDE)
    names = [c for c in cols_s if c != "key"]
    for s0 in range(start, start + rows, chunk):
        m = min(chunk, start + rows - s0)
        cols = synth.config_c(m, start=s0)
        keys = pa.array([f"key{i}" for i in range(s0, s0 + m)], pa.string())
        rt.write(pa.RecordBatch.from_arrays([keys] + [synth.to_arrow(c) for c in cols], names=["key"] + names))
    return rt, names


def verify_arrays(ctx, seg, proj, outs, b, host_blob, host_off, want=None):
    """Decoded block b (device) against the oracle's decode of its host bytes,
    bit for bit (the comparator of tests/golden_util.assert_array_equal).
    Returns a list of mismatch descriptions (empty = identical)."""
    from murr_amd.device import download_array
    if want is None:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        want = O.decode_block(O.Segment([int(c.dtype) for c in seg.columns]), proj, host_blob, host_off)
    n = host_off.size - 1
    bad = []
    for p, ci in enumerate(proj):
        e = want[p]
        g = download_array(ctx, outs.array(b, p), int(seg.columns[ci].dtype), n)
        nb = (n + 7) // 8
        if g["null_count"] != e["null_count"]:
            bad.append(f"block {b} col {p}: null_count")
        elif e["validity"] is not None and bytes(g["validity"][:nb]) != e["validity"]:
            bad.append(f"block {b} col {p}: validity")
        dt = e["dtype"]
        if dt == 0:
            if not np.array_equal(np.asarray(g["offsets"][: n + 1], np.int32), e["offsets"]):
                bad.append(f"block {b} col {p}: offsets")
            elif bytes(g["values"][: int(e["offsets"][-1])]) != e["values"]:
                bad.append(f"block {b} col {p}: utf8 data")
        elif dt == 1:
            if bytes(g["values"][:nb]) != e["values"]:
                bad.append(f"block {b} col {p}: bool bits")
        elif bytes(g["values"][: len(e["values"])]) != e["values"]:
            bad.append(f"block {b} col {p}: values")
    return bad, want


def run_decode(args, dist, rank, world, local_rank):
    check_gpus(local_rank, world)
    ctx = Context(local_rank)
    rows, K = args.rows, args.blocks
    if args.table_rows:
        # configs[3] as written: ONE table of --table-rows rows split by key
        # range over the ranks (strong scaling: rank r decodes its range)
        start, rows = shard_rows(rank, world, args.table_rows)
    else:
        start, _ = shard_rows(rank, world, rows * world)  # weak scaling: `rows` per rank
    rt = None
    t_build = time.perf_counter()
    if args.config == "D":
        # config D: this rank's key-range shard as a resident table; one step =
        # ResidentTable.scan_device, the whole shard in one launch cut on the
        # table's own utf8 index (kept by every write)
        K = 1
        rt, names = config_d_table(ctx, rows, start, stride=args.resident_stride)
        seg = rt.segment
        proj = parse_proj(args.proj, len(seg.columns))
        blocks = [rt.block()]
        ix_stride = blocks[0].stride
    else:
        cols = make_columns(args.config, rows, start=start)
        seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
        proj = parse_proj(args.proj, len(cols))
        dcols = synth.upload_columns(ctx, cols)
        if args.uidx_stride:
            # the block and its utf8 index, written together (murr_encode_batch_ix)
            b0 = encode_block(ctx, seg, dcols, rows, args.uidx_stride)
        else:
            dblob, doff, blen = encode_batch(ctx, seg, dcols, rows)
            b0 = DeviceBlock(dblob, doff, rows, blen)
        del dcols
        if args.offsets == 32:
            # u32 block-relative row offsets (murr_block_t.row_off32): a
            # 100k-row block is 1.8 MB, far below 4 GiB
            b0 = b0.narrow(ctx)
        if args.arena:  # K resident blocks in arenas (blobs / row offsets / outputs each one buffer)
            blocks = arena_blocks(ctx, b0, K, args.arena)
        else:
            blocks = [b0] + [copy_block(ctx, b0) for _ in range(K - 1)]  # K resident blocks
        ix_stride = b0.stride
    ctx.sync()
    build_s = time.perf_counter() - t_build
    host_blob = blocks[0].data.download(blocks[0].data_bytes)
    host_off = blocks[0].host_offsets()
    ix_bytes = 8 * int(L_len(ctx, seg, rows, ix_stride)) if blocks[0].uidx is not None else 0
    # Output sets: step s decodes into set s % n_sets and is launched
    # (murr_decode_run_async) before step s - 1 is waited for, so the host's
    # launch and read-back work overlaps the previous step's kernel, as a
    # serving loop would.  One lane: two sets on one context (one stream; on
    # the GPU the steps run one after the other).  L > 1 lanes: one set per
    # lane, each lane a context of its own (its own stream), L - 1 steps
    # launched ahead, so step s + 1's workgroups can start on CUs step s has
    # left.  --sync-steps: one set, each step waited for (the A/B).
    #
    # Lane policy, the same for every config: the headline
    # line is per launch -- one lane, so the roofline's kernel time and a
    # rocprof trace's kernel duration describe one launch's traffic -- and the
    # overlapped rate is an extra key (`lanes`: --extra-lanes L, default 3;
    # config D's shard scan and config B both gain from it), measured after
    # the headline with every lane's last output checked against the oracle.
    names = [seg.columns[c].name for c in proj] if rt is not None else None
    every = _abi.PLAN_TIME_EVERY
    if "MURR_TIME_EVERY" in os.environ and _abi.LIB_PATH.endswith("_tuning.so"):
        every = max(1, int(os.environ["MURR_TIME_EVERY"]))

    def lanes_run(nl, steps, warmup):
        """Warm-up + timed region over nl lanes; returns the region's state."""
        # one output set per lane (two on one context with one lane); step s
        # uses set s % len(ctxs), and len(ctxs) - 1 steps are launched ahead
        # of the one waited for
        ctxs = [ctx] + [Context(local_rank) for _ in range(nl - 1)] if nl > 1 else [ctx, ctx]
        if args.arena:
            out_sets = [ArenaOutputs(c, seg, proj, blocks, args.arena) for c in ctxs]
        else:
            out_sets = [DecodeOutputs(c, seg, proj, blocks) for c in ctxs]
        plans = None
        if rt is not None:
            def launch(i):  # the product call (its prepared plan after the first)
                return rt.scan_device_async(names, out_sets[i], ctx=ctxs[i])
        else:
            # the launch prepared once per output set (murr_decode_plan)
            plans = [DecodePlan(c, seg, proj, blocks, o) for c, o in zip(ctxs, out_sets)]

            def launch(i):
                plans[i].run_async()
                return plans[i]

        # Kernel time.  The warm-up samples the plan's own timed runs (one in
        # PLAN_TIME_EVERY, the first included).  The timed region turns those
        # per-run events off (each costs GPU time between back-to-back
        # launches) and brackets all K launches with two marks on the context's
        # stream: kernel_ms_avg = that GPU time / K, which includes the gaps
        # between the launches, so it never exceeds ms_per_step (the host's
        # clock around the same K steps).  With several lanes (streams) the
        # region runs from the first lane's start mark to the latest of the
        # lanes' end marks: the launches overlap, so this is the GPU time per
        # launch at steady state.
        runs = [0] * len(ctxs)  # runs of each output set's plan so far
        launched = {}  # the prepared plans the steps ran (resident scans make theirs inside the table)

        def run_steps(n, sample=True):
            ms = []

            def done(i):
                if sample and runs[i] % every == 0:
                    ms.append(ctxs[i].last_kernel_ms())
                runs[i] += 1

            def go(i):
                p = launch(i)
                launched[id(p)] = p
                return p

            if args.sync_steps:
                for _ in range(n):
                    go(0).wait()
                    done(0)
                return ms
            nset = len(ctxs)
            inflight = [go(s % nset) for s in range(min(n, nset - 1))]
            for s in range(n):
                if s + nset - 1 < n:
                    inflight.append(go((s + nset - 1) % nset))
                inflight.pop(0).wait()
                done(s % nset)
            return ms

        if rt is not None:
            # setup: a resident table prepares each lane's scan plan at its
            # first scan; make those before the warm-up, so a warm-up shorter
            # than the lane count cannot leave one to the timed region
            for i in range(len(ctxs)):
                launch(i).wait()
        wms = run_steps(warmup)
        for p in launched.values():
            p.time_every(0)
        lanes = list({id(c): c for c in ctxs}.values())
        barrier(dist)
        for c in ctxs:
            c.sync()
        t0 = time.perf_counter()
        ctx.mark(0)
        run_steps(steps, sample=False)
        for c in lanes:
            c.mark(1)
        for c in ctxs:
            c.sync()
        barrier(dist)
        elapsed = time.perf_counter() - t0
        region_ms = max(ctx.mark_ms(0, 1, c) for c in lanes) if steps else None
        for p in launched.values():
            p.time_every(every)
        nset = 1 if args.sync_steps else len(ctxs)
        # the set each lane's last timed step wrote (step s used set s % nset)
        last_of = {i: max(s for s in range(steps) if s % nset == i) for i in range(min(nset, steps))}
        return {"ctxs": ctxs, "lanes": lanes, "out_sets": out_sets, "plans": plans, "launch": launch,
                "elapsed": elapsed, "region_ms": region_ms, "wms": wms, "last_of": last_of,
                "last": (steps - 1) % nset if steps else 0}

    R = lanes_run(1 if args.lanes is None else args.lanes, args.steps, args.warmup)
    ctxs, out_sets, plans, launch = R["ctxs"], R["out_sets"], R["plans"], R["launch"]
    elapsed, region_ms, wms, last = R["elapsed"], R["region_ms"], R["wms"], R["last"]
    outs = out_sets[last]  # the last timed step's output (checked below)
    elapsed = max_over_ranks(dist, elapsed)
    stats = ctx.stats()

    a0 = [outs.array(0, p) for p in range(len(proj))]
    out_block = arrow_out_bytes(seg, proj, rows, [a.null_count for a in a0],
                                [a.data_len for a in a0])
    off_w = blocks[0].offset_width  # u32 (row_off32) or u64 row offsets
    in_block = int(host_blob.size) + off_w * (rows + 1) + ix_bytes  # blobs, row offsets, utf8 index
    out_step = out_block * K
    total_out = sum_over_ranks(dist, out_step * args.steps)
    value = total_out / elapsed / GIB
    warm_ms = wms[1:] or wms  # (the very first run pays one-off costs)
    if region_ms is not None:
        k_avg_ms = region_ms / args.steps
    else:
        k_avg_ms = float(np.mean(warm_ms))  # (no timed steps: the warm-up's sampled runs)
    achieved = (in_block + out_block) * K / (k_avg_ms * 1e-3) / 1e9
    shape = "%dx%d" % tuple(stats["last_shape"])
    timed_kernel = ("decode_kernel" if stats["last_mode"] == "generic" else
                    "murr_jit_decode_%s%s" % ("split_" if stats["last_mode"] == "split" else "", shape))
    traffic = pmc_traffic(args.pmc_csv, timed_kernel)
    if traffic is None and not args.pmc_csv and not args.no_traffic and world == 1 and rank == 0:
        traffic = measure_traffic(args, timed_kernel)

    # after the timed region: the timed launch's output, checked against the
    # oracle (first and last block); a mismatch fails the run
    checked = sorted({0, K - 1}) if not args.no_verify else []
    bad, want = [], None
    for b in checked:
        bb, want = verify_arrays(ctx, seg, proj, outs, b, host_blob, host_off, want)
        bad += bb
    if bad:
        raise SystemExit("bench: decoded output differs from the oracle: " + "; ".join(bad[:8]))
    # the same launch without the utf8 index (untimed variant, for DESIGN.md)
    no_index_ms = None
    if ix_bytes:
        bare = [DeviceBlock(b.data, b.row_off, b.n_rows, b.data_bytes, row_off32=b.row_off32) for b in blocks]
        p2 = DecodePlan(ctx, seg, proj, bare, outs)
        nk = []
        for r in range(5 * every):
            p2.run()
            if r % every == 0:
                nk.append(ctx.last_kernel_ms())
        no_index_ms = round(float(np.mean(nk[1:])), 5)
        p2.close()
        # leave the indexed output in place
        launch(last).wait()
    # the overlapped rate (lane policy above): --extra-lanes contexts, every
    # lane's last timed output checked against the oracle
    lanes_extra = None
    if args.extra_lanes > 1 and (args.lanes or 1) == 1 and args.steps:
        E = lanes_run(args.extra_lanes, args.steps, args.warmup)
        el = max_over_ranks(dist, E["elapsed"])
        ebad = []
        for i in sorted(E["last_of"]):
            for b in checked:
                bb, want = verify_arrays(E["ctxs"][i], seg, proj, E["out_sets"][i], b, host_blob, host_off, want)
                ebad += [f"lane {i}: {x}" for x in bb]
        if ebad:
            raise SystemExit("bench: a lane's output differs from the oracle: " + "; ".join(ebad[:8]))
        lanes_extra = {
            "lanes": args.extra_lanes, "value": round(total_out / el / GIB, 3),
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "frac_step_lanes": round((in_block + out_block) * K / (el / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
            "gpu_ms_per_step": round(E["region_ms"] / args.steps, 5),
            "verified": (f"every lane's last timed output, blocks {checked}, bit-exact vs the oracle" if checked
                         else "NOT VERIFIED (--no-verify)"),
            "note": "launches on separate streams overlap: a per-launch roofline does not apply"}
        for pl in E["plans"] or []:
            pl.close()
        for c in E["ctxs"][1:]:
            c.close()
        del E
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if args.table_rows else "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": {"B": "configs[1] read_block shape: 100k-row FLOAT32+UTF8 blocks",
                                "C": "configs[2] schema: 16-col mixed nullable blocks",
                                "D": "configs[3] shard: 16-col mixed nullable, key-range shard per GPU, "
                                     "ResidentTable.scan"}.get(args.config, args.config),
                   "rows_per_block": rows, "blocks_per_step": K, "columns": len(proj),
                   "table_rows": args.table_rows or None,
                   "rows_per_rank": [shard_rows(r, world, args.table_rows)[1] for r in range(world)]
                   if args.table_rows else [rows] * world,
                   "utf8_index_stride": ix_stride if ix_bytes else None,
                   "row_offset_bytes": off_w,
                   "bytes_in_per_step": in_block * K, "bytes_out_per_step": out_step,
                   "parallelism": f"{world} key-range shard(s), no collective",
                   "launch": {"mode": stats["last_mode"], "grid": stats["last_grid"],
                              "shape": "%dx%d" % stats["last_shape"], "split_retries": stats["split_retries"]},
                   "setup_s": round(build_s, 2)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     # the same bytes over the driver-visible step (host clock)
                     "frac_step": round((in_block + out_block) * K / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": ctx.last_kernel(),
                     "kernel_ms_avg": round(k_avg_ms, 5),
                     "kernel_ms_timing": "GPU marks around the timed region / steps" if region_ms is not None
                     else "mean of the plans' timed runs",
                     "kernel_ms_sampled_warmup": round(float(np.mean(warm_ms)), 5) if warm_ms else None,
                     "algorithmic_bytes_per_launch": (in_block + out_block) * K},
        "verified": f"blocks {checked} of the timed launch bit-exact vs the oracle" if checked else "NOT VERIFIED (--no-verify)",
        "no_index_ms": no_index_ms,
        "lane_policy": ("per launch: one stream, steps back to back; the overlapped rate of "
                        f"{args.extra_lanes} streams is `lanes`" if (args.lanes or 1) == 1 else
                        f"{args.lanes} lanes (tuning run)"),
        "lanes": lanes_extra,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(seg, proj, host_blob, host_off, rows, args.cpu_seconds)
        threads, src = host_cores()
        if threads > 1:
            line["cpu_baseline_all_cores"] = cpu_baseline_threads(seg, proj, host_blob, host_off, rows,
                                                                  min(5.0, args.cpu_seconds), threads)
            line["cpu_baseline_all_cores"]["cores_source"] = src
    if rank == 0:
        print(json.dumps(line), flush=True)
    if rt is None:
        for pl in plans:
            pl.close()
    del rt
    ctx.close()


def run_harness(args, dist, rank, world, local_rank):
    """Self-test of the multi-rank harness (spawner, barriers, max/sum over
    ranks, the JSON line) without a GPU: the "step" copies a host buffer.
    Never a measurement: data = "harness self-test"."""
    rows = None
    if args.table_rows:  # the row split of configs[3] as written (strong scaling)
        _, rows = shard_rows(rank, world, args.table_rows)
    buf = np.zeros(max(rows or 0, 1 << 20) if rows is None else max(rows, 1), np.uint8)
    dst = np.empty_like(buf)
    for _ in range(args.warmup):
        np.copyto(dst, buf)
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.copyto(dst, buf)
    barrier(dist)
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    total = sum_over_ranks(dist, float(buf.nbytes * args.steps))
    rows_all = sum_over_ranks(dist, float(rows or 0))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(total / elapsed / GIB, 3), "unit": "GiB/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "strong" if args.table_rows else "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "harness self-test",
                          "config": {"workload": "host memcpy (harness test only)",
                                     "table_rows": args.table_rows or None,
                                     "rows_per_rank": [shard_rows(r, world, args.table_rows)[1] for r in range(world)]
                                     if args.table_rows else None,
                                     "rows_summed_over_ranks": int(rows_all) if args.table_rows else None,
                                     "parallelism": f"{world} rank(s)"}}), flush=True)


def host_arrow_bytes(outs, nproj):
    """Arrow bytes of one batch's host arrays (SURVEY.md §8(d) bytes_out)."""
    tot = 0
    for p in range(nproj):
        h = outs[p]
        tot += h.values_len + (4 * (h.length + 1) if h.offsets else 0) + ((h.length + 7) // 8 if h.validity else 0)
    return tot


def run_host(args):
    """PCIe-inclusive rate (north_star: host memory in, host memory out), two ways:
      stream   murr_hstream (ReadBatchBuilder batches back to back, pipelined
               over --depth slots: H2D of batch i+1 || decode of i || D2H of
               i-1), --blocks K batches after --warmup, from a ring of
               --host-ring distinct blocks held in pinned memory (a block
               cache allocated with murr_host_alloc) and, as a second line,
               from pageable memory (one host memcpy into pinned staging per
               batch);
      builder  the serial one-batch path (murr_builder_*: H2D, decode, D2H on
               one stream), the round-3 number.
    Every block's arrays are checked against the oracle for the first and the
    last batch of each run."""
    from murr_amd.row import HostBuffer, HostStream, ReadBatchBuilder, host_array_buffers
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    ctx = Context(0)
    rows = args.rows
    ring = max(1, min(args.host_ring, args.blocks))
    blocks = []
    for r in range(ring):
        cols = make_columns(args.config, rows, r * rows)
        seg = SegmentSchema([(f"c{i}", c["dtype"]) for i, c in enumerate(cols)])
        dblob, doff, blen = encode_batch(ctx, seg, synth.upload_columns(ctx, cols), rows)
        blocks.append((dblob.download(blen), doff.download((rows + 1) * 8).view(np.uint64).copy()))
        del dblob, doff
    proj = list(range(len(seg.columns)))
    oseg = O.Segment([int(c.dtype) for c in seg.columns])
    want = {}
    # the row offsets the batches carry: u32 (murr_hstream_submit32, half the
    # offset bytes over PCIe) or u64 (--offsets)
    odt = np.uint32 if args.offsets == 32 else np.uint64
    src_off = [off.astype(odt) for _, off in blocks]
    # the pinned block cache: every ring block copied once into murr_host_alloc memory
    pinned = []
    for (blob, _), off in zip(blocks, src_off):
        hb, ho = HostBuffer(blob.size + 16, ctx), HostBuffer(off.nbytes, ctx)
        hb.array[: blob.size] = blob
        ho.array[:] = off.view(np.uint8)
        pinned.append((hb, ho, ho.array.view(odt)))

    def check(outs, r):
        if r not in want:
            want[r] = O.decode_block(oseg, proj, blocks[r][0], blocks[r][1])
        for p in range(len(proj)):
            g, e = host_array_buffers(outs[p]), want[r][p]
            ok = g["null_count"] == e["null_count"] and (e["validity"] is None or g["validity"] == e["validity"])
            if e["dtype"] == 0:
                ok = ok and np.array_equal(g["offsets"], e["offsets"]) and g["values"] == e["values"]
            else:
                ok = ok and g["values"][: len(e["values"])] == e["values"]
            if not ok:
                raise SystemExit(f"bench host: batch of ring block {r} col {p} differs from the oracle")

    def stream_run(use_pinned):
        hs = HostStream(seg, proj, depth=args.depth, ctx=ctx)
        total = args.warmup + args.blocks
        out_bytes, t0, done = 0, None, 0

        def submit(i):
            r = i % ring
            if use_pinned:
                hb, _, off = pinned[r]
                hs.submit(hb.array, off, pinned=True)
            else:
                hs.submit(blocks[r][0], src_off[r])

        nxt = 0
        while nxt < min(args.depth, total):
            submit(nxt)
            nxt += 1
        tail = []  # the last `depth` batches: their slots are not reused after the loop
        while done < total:
            if done == args.warmup:
                st0 = hs.stats()
                t0 = time.perf_counter()
            outs = hs.next()
            i = done
            done += 1
            if i >= args.warmup:
                out_bytes += host_arrow_bytes(outs, len(proj))
                if i >= total - args.depth:
                    tail.append((outs, i % ring))
            if nxt < total:
                submit(nxt)
                nxt += 1
        el = time.perf_counter() - t0
        st1 = hs.stats()
        # checked after the timed region: the last `depth` timed batches, whose
        # pinned outputs stay in place once nothing more is submitted
        for outs, r in tail:
            check(outs, r)
        hs.close()
        d = {k: st1[k] - st0[k] for k in st1}
        nb, nt = d["batches"], max(d["timed_batches"], 1)  # (copies and kernel timed on every eighth batch)
        h2d_b, d2h_b = d["h2d_bytes"] / nb, d["d2h_bytes"] / nb
        return {"GiB_s_host_to_host": round(out_bytes / el / GIB, 3),
                "ms_per_batch": round(el / args.blocks * 1e3, 4),
                "arrow_bytes_out_per_batch": out_bytes // args.blocks,
                "h2d_GB_s": round(h2d_b / (d["h2d_ms"] / nt * 1e-3) / 1e9, 2) if d["h2d_ms"] else None,
                "d2h_GB_s": round(d2h_b / (d["d2h_ms"] / nt * 1e-3) / 1e9, 2) if d["d2h_ms"] else None,
                "h2d_ms_per_batch": round(d["h2d_ms"] / nt, 4), "kernel_ms_per_batch": round(d["kernel_ms"] / nt, 4),
                "d2h_ms_per_batch": round(d["d2h_ms"] / nt, 4),
                "host_submit_ms_per_batch": round(d["host_submit_ms"] / nb, 4),
                "host_next_ms_per_batch": round(d["host_next_ms"] / nb, 4),
                "host_wait_ms_per_batch": round(d["host_wait_ms"] / nb, 4),
                "h2d_bytes_per_batch": int(h2d_b), "d2h_bytes_per_batch": int(d2h_b)}

    res = {"pinned_source": stream_run(True), "pageable_source": stream_run(False)}
    # the serial builder path (round 3's number): one batch at a time, rows added one by one
    blob, off = blocks[0]
    tm = []
    for it in range(max(2, min(args.warmup, 3)) + min(args.steps, 20)):
        b = ReadBatchBuilder(seg, seg.columns, rows, ctx)
        ptrs = (C.c_void_p * rows)()
        lens = (C.c_uint64 * rows)()
        base = blob.ctypes.data
        ptrs[:] = (base + off[:-1].astype(np.int64)).tolist()
        lens[:] = np.diff(off).tolist()
        ctx.L.murr_builder_add_rows(b.h, ptrs, lens, rows)
        outs = b._build_host()
        if it >= 2:
            tm.append(b.last_timing())
    obytes = host_arrow_bytes(outs, len(proj))
    med = {k: float(np.median([t[k] for t in tm])) for k in tm[0]}
    res["builder_serial"] = {"median_ms": med, "GiB_s_pcie_inclusive": round(obytes / (med["total_ms"] * 1e-3) / GIB, 3)}
    print(json.dumps({"mode": "host", "config": args.config, "rows_per_batch": rows, "batches": args.blocks,
                      "warmup": args.warmup, "depth": args.depth, "ring_blocks": ring,
                      "blob_bytes_per_batch": int(blocks[0][0].size), "row_offset_bytes": args.offsets // 8,
                      "verified": f"the last {args.depth} timed batches of each streaming run bit-exact vs the "
                      "oracle, checked after the timed region", **res}))


def run_encode(args):
    """configs[4] write shape: Arrow (10 x f32) -> row blobs, device-resident."""
    ctx = Context(0)
    n = args.rows
    cols = make_columns(args.enc_config, n, 0)
    seg = SegmentSchema([(f"col_{i}", c["dtype"]) for i, c in enumerate(cols)])
    dcols = synth.upload_columns(ctx, cols)
    # one output allocation reused by every step (a write path keeps its
    # arena; allocating ~1 GB per call would time the allocator, not the encode)
    out = encode_batch(ctx, seg, dcols, n)[:2]
    for _ in range(args.warmup):
        encode_batch(ctx, seg, dcols, n, out=out)
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        blob, off, blen = encode_batch(ctx, seg, dcols, n, out=out)
        kms.append(ctx.last_kernel_ms())
    el = time.perf_counter() - t0
    bytes_in = sum(c["values"].nbytes + (c["offsets"].nbytes if c["offsets"] is not None else 0)
                   + (c["validity"].nbytes if c["validity"] is not None else 0) for c in cols)
    bytes_out = blen + 8 * (n + 1)
    k = float(np.mean(kms))
    print(json.dumps({"mode": "encode", "config": args.enc_config, "kernel": ctx.last_kernel(), "rows": n, "bytes_in": bytes_in, "bytes_out": bytes_out,
                      "kernel_ms_avg": round(k, 4), "ms_per_step": round(el / args.steps * 1e3, 3),
                      "recounts": ctx.stats()["encode_recounts"],
                      "GB_s_algorithmic": round((bytes_in + bytes_out) / (k * 1e-3) / 1e9, 1),
                      "frac_of_8TBs": round((bytes_in + bytes_out) / (k * 1e-3) / 8e12, 4),
                      "GiB_s_blob_out": round(bytes_out / (k * 1e-3) / GIB, 2)}))


def resident_table(ctx, kind: str, n: int, chunk: int = 10_000_000):
    """A ResidentTable of n rows, written in chunks (ResidentTable.write appends).
    kind "C": config C's 16 mixed nullable columns, keys "key{i}";
    kind "ref": the reference bench dataset (benches/common/dataset.rs:24-55):
    col_0..col_9 float32 = i, key = i.to_string()."""
    import pyarrow as pa
    from murr_amd import ColumnSchema, TableSchema
    from murr_amd.resident import ResidentTable
    if kind == "ref":
        ts = synth.ref_schema()
    else:
        cols_s = {"key": ColumnSchema(D.Utf8, False)}
        cols_s.update({f"c{i}": ColumnSchema(c["dtype"]) for i, c in enumerate(synth.config_c(1))})
        ts = TableSchema("key", cols_s)
    rt = ResidentTable(ts, ctx)
    names = [c for c in ts.columns if c != "key"]
    for start in range(0, n, chunk):
        m = min(chunk, n - start)
        if kind == "ref":
            rt.write(synth.ref_batch(start, m))
            continue
        cols = synth.config_c(m, start=start)
        keys = pa.array([f"key{i}" for i in range(start, start + m)], pa.string())
        rt.write(pa.RecordBatch.from_arrays([keys] + [synth.to_arrow(c) for c in cols], names=["key"] + names))
    return rt, names


def ref_keys(kind: str, rows: int, nq: int, k: int):
    """Key set k of a bench: kind "ref" samples like run_read_bench
    (benches/common/read_bench.rs:89-98: seed num_keys * 2_000_000 + k, uniform
    over [0, rows), key = i.to_string(); numpy's generator in place of rand's
    StdRng, so the same distribution, not the same keys); kind "C" draws over
    1.05 x rows, so about 5 % miss."""
    if kind == "ref":
        ids = np.random.default_rng(nq * 2_000_000 + k).integers(0, rows, size=nq)
        return [str(int(i)) for i in ids]
    ids = np.random.default_rng(44 + k).integers(0, int(rows * 1.05), size=nq)
    return [f"key{int(i)}" for i in ids]


def resident_cpu_baseline(rt, kind: str, n: int, names, qarr, reads: int):
    """CPU baseline of a resident read: the oracle's MemoryStore restatement
    (src/io/store/memory.rs:28-45: a key map, then ReadBatchBuilder add_row /
    add_empty per key and build) over the same table's keys and blobs (the
    arena downloaded), the same key sets, one host thread.  None above 20 M
    rows (the host key map of read_block's 100 M rows is not a bounded
    sample)."""
    if n > 20_000_000:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import pyarrow as pa
    blob = rt.arena.download(max(rt.used, 1))
    off = rt.row_off.download(8 * (rt.n + 1)).view(np.uint64)
    keys = pa.array([str(i) for i in range(n)] if kind == "ref" else [f"key{i}" for i in range(n)], pa.string())
    store = O.MemStore(keys, blob, off)
    seg = O.Segment([int(c.dtype) for c in rt.segment.columns])
    proj = [c.index for c in rt._resolve(names)]
    pj = (C.c_uint32 * len(proj))(*proj)
    outs = (O.OcArray * len(proj))()
    err = O.OcError()
    bufs = [(q.buffers(), len(q)) for q in qarr]

    def once(i):
        qb, nq = bufs[i % len(bufs)]
        t0 = time.perf_counter()
        st = store.read_raw(seg, pj, len(proj), qb[2].address, qb[1].address, nq, outs, err)
        dt = time.perf_counter() - t0
        assert st == 0, st
        for p in range(len(proj)):
            O.lib().oc_array_free(C.byref(outs[p]))
        return dt

    for i in range(5):
        once(i)
    ts = [once(i) for i in range(reads)]
    store.close()
    return {"us_per_read_median": round(float(np.median(ts)) * 1e6, 1), "cores": 1, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{reads} reads of the same key sets through oracle/libmurr_oracle.so oc_memstore_read "
                      f"(MemoryStore restatement, FNV map in place of SipHash) over the table's {n} rows"}


def run_resident(args):
    """Device-resident Table::read on a table of
    args.rows rows in HBM: `--table C` (config C) or `--table ref` (the
    reference read benches' dataset: --rows 100000000 is benches/read_block.rs,
    10000000 benches/read_plain.rs).  `--keys` keys per read.  Two timings,
    medians over --steps reads on rotating key sets:
      device: lookup + gather (murr_index_gather) + decode (murr_decode_blocks),
        keys already in HBM, no host round trip (host-synchronous wall time);
      host: ResidentTable.read, keys from Python to a RecordBatch on the host
        (what benches/common/read_bench.rs times around Table::read)."""
    import pyarrow as pa
    from murr_amd.resident import _upload_utf8
    ctx = Context(0)
    n, nq = args.rows, args.keys
    t0 = time.perf_counter()
    rt, names = resident_table(ctx, args.table, n)
    build_s = time.perf_counter() - t0
    seg = rt.segment
    qsets = [ref_keys(args.table, n, nq, k) for k in range(4)]
    dq = [_upload_utf8(ctx, pa.array(q, pa.string())) for q in qsets]
    cap = max(nq * rt.max_row, 16)
    data, roff, needed = ctx.alloc(cap + 16), ctx.alloc((nq + 1) * 8), ctx.alloc(8)
    blk = DeviceBlock(data, roff, nq, min(cap, max(16, int(rt.used / max(rt.n, 1) * nq))))
    proj = list(range(len(seg.columns)))
    outs = DecodeOutputs(ctx, seg, proj, [blk])
    cb = (_abi.Block * 1)()
    cb[0].data, cb[0].row_off, cb[0].n_rows, cb[0].data_bytes = data.ptr, roff.ptr, nq, blk.data_bytes
    pj = (C.c_uint32 * len(proj))(*proj)
    err = _abi.Error()
    L = ctx.L

    def read_unprepared(q):  # (round 5's path: two calls, descriptors uploaded per read)
        st = L.murr_index_gather(ctx.h, rt.index.h, q[0].ptr, q[1].ptr, nq, rt.arena.ptr, rt.row_off.ptr,
                                 data.ptr, cap, roff.ptr, None, needed.ptr)
        assert st == 0, st
        st = L.murr_decode_blocks(ctx.h, C.byref(seg.c), pj, len(proj), cb, 1, outs.arrays, C.byref(err))
        assert st == 0, (st, err.status)

    # the product path: the table's prepared read (ReadPlan: lookup + gather +
    # decode enqueued once, one wait), keys already in HBM
    rplan = rt.read_plan(names, nq)
    assert rplan is not None, "read too large for a prepared read"

    def read(q):
        rplan.run_device(q[0].ptr, q[1].ptr, nq)

    def timed(fn, n):
        for i in range(args.warmup):
            fn(dq[i % 4])
        t = []
        for i in range(n):
            t0 = time.perf_counter()
            fn(dq[i % 4])
            t.append(time.perf_counter() - t0)
        return t

    ts = timed(read, args.steps)
    tu = timed(read_unprepared, args.steps)
    # the prepared read's output against the unprepared path's (same keys): bit for bit
    from murr_amd.device import download_array
    read(dq[0])
    read_unprepared(dq[0])
    for p, ci in enumerate(proj):
        dt = int(seg.columns[ci].dtype)
        a, b = download_array(ctx, rplan.dev_outs[p], dt, nq), download_array(ctx, outs.array(0, p), dt, nq)
        assert a["null_count"] == b["null_count"] and a["values"] == b["values"], f"column {p}"
        assert (a["offsets"] is None and b["offsets"] is None) or np.array_equal(a["offsets"], b["offsets"])
    for i in range(args.warmup):
        rt.read(qsets[i % 4], names)
    th = []
    for i in range(args.steps):
        t0 = time.perf_counter()
        rb = rt.read(qsets[i % 4], names)
        th.append(time.perf_counter() - t0)
    out_bytes = sum(sum(b.size for b in col.buffers() if b is not None) for col in rb.columns)
    # the same reads with the keys already an Arrow array (what an Arrow-native
    # caller -- the Rust binding of INTEGRATION.md -- hands over): the library
    # run + the RecordBatch, without Python's list -> Arrow conversion
    qarr = [pa.array(q, pa.string()) for q in qsets]
    for i in range(args.warmup):
        rt.read(qarr[i % 4], names)
    ta = []
    for i in range(args.steps):
        t0 = time.perf_counter()
        rt.read(qarr[i % 4], names)
        ta.append(time.perf_counter() - t0)
    cpu_read = None if args.no_cpu else resident_cpu_baseline(rt, args.table, n, names, qarr, min(args.steps, 200))
    hplan = rt.read_plan(names, nq)  # the library call alone (arrays left in pinned memory)
    tr = []
    for i in range(args.steps):
        t0 = time.perf_counter()
        hplan.run(qarr[i % 4])
        tr.append(time.perf_counter() - t0)
    ipc_res = {}
    if args.ipc:
        # + Arrow IPC record-batch message packed in HBM (murr_ipc_batch_device)
        # and one D2H into pinned memory: the HTTP fetch handler's StreamWriter
        # body (src/api/http/handlers.rs:93-101) ready for the socket.
        mlen = C.c_uint64()
        read(dq[0])
        st = L.murr_ipc_batch_device(ctx.h, C.byref(seg.c), pj, len(proj), rplan.dev_outs, nq, 64, None, 0,
                                     C.byref(mlen), C.byref(err))
        assert st == 0, st
        mcap = int(mlen.value) + 4096 * len(proj)  # body sizes vary a little with the key set
        dmsg = ctx.alloc(mcap)
        hmsg = C.c_void_p()
        assert L.murr_host_alloc(ctx.h, mcap, C.byref(hmsg)) == 0

        def read_ipc(q):
            read(q)
            st = L.murr_ipc_batch_device(ctx.h, C.byref(seg.c), pj, len(proj), rplan.dev_outs, nq, 64, dmsg.ptr,
                                         mcap, C.byref(mlen), C.byref(err))
            assert st == 0, (st, err.required)
            assert L.murr_memcpy_d2h(ctx.h, hmsg, dmsg.ptr, mlen.value) == 0

        for i in range(args.warmup):
            read_ipc(dq[i % 4])
        ti = []
        for i in range(args.steps):
            t0 = time.perf_counter()
            read_ipc(dq[i % 4])
            ti.append(time.perf_counter() - t0)
        L.murr_host_free(ctx.h, hmsg)
        ipc_res = {"ipc_message_bytes": int(mlen.value),
                   "us_per_read_ipc_median": round(float(np.median(ti)) * 1e6, 1),
                   "ipc_path": "gather + decode + ipc_pack + one D2H (pinned)"}
    med = float(np.median(ts))
    shape = {100_000_000: "benches/read_block.rs", 10_000_000: "benches/read_plain.rs"}.get(n, "")
    print(json.dumps({"mode": "resident", "table": args.table, "bench_shape": shape if args.table == "ref" else "",
                      "table_rows": n, "keys_per_read": nq, "columns": len(proj), "build_s": round(build_s, 2),
                      "arrow_bytes_out": out_bytes,
                      "us_per_read_device_median": round(med * 1e6, 1),
                      "us_per_read_device_p95": round(float(np.percentile(ts, 95)) * 1e6, 1),
                      "device_path": "ReadPlan.run_device: fused probe + look-back + gather copy, prepared decode; one wait",
                      "us_per_read_device_unprepared_median": round(float(np.median(tu)) * 1e6, 1),
                      "us_per_read_host_median": round(float(np.median(th)) * 1e6, 1),
                      "us_per_read_host_arrow_keys_median": round(float(np.median(ta)) * 1e6, 1),
                      "us_per_read_host_plan_run_median": round(float(np.median(tr)) * 1e6, 1),
                      "cpu_baseline": cpu_read,
                      "GiB_s_arrow_out_device": round(out_bytes / med / GIB, 3),
                      "host_path": "ResidentTable.read: Python keys -> Arrow -> ReadPlan.run -> RecordBatch",
                      "kernels": "gather_fused, murr_jit_decode (+ copy_segs_kernel on the host path)",
                      **ipc_res}))


def sst_blocks(rows: int, comp: int, block_size: int = 512):
    """The SST data blocks the reference's store would hold for the read
    benches' dataset (keys i.to_string(), 10 x f32 row blobs), in key order,
    cut at block_size with restart interval 8 and BinaryAndHash
    (src/io/store/rocksdb/block.rs:83-111); blocks stored with `comp`."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
    import sstgen as G
    ctx = Context(0)
    rt, _ = resident_table(ctx, "ref", rows)
    arena = rt.arena.download(rt.used).tobytes()
    off = rt.row_off.download(8 * (rows + 1)).view(np.uint64)
    order = sorted(range(rows), key=lambda i: str(i))
    entries = [(str(i).encode(), rows + i, G.TYPE_VALUE, arena[off[i]:off[i + 1]]) for i in order]
    return [(G.compress(b, comp), comp) for b in G.blocks_of(entries, block_size=block_size)]


def run_sst(args):
    """§8(f) rank 4: a whole SST's data blocks (resident in HBM) -> entries in
    HBM (murr_sst_decode: inflate, count, scans, entry decode).  Wall time per
    call (host-synchronous, the library's output allocations included) and the
    entry-decode kernel's event time; rates over the stored bytes read plus the
    entry bytes written."""
    from murr_amd import sst
    comp = {"none": 0, "snappy": 1, "lz4": 4}[args.sst_compression]
    t0 = time.perf_counter()
    stored = sst_blocks(args.rows, comp)
    gen_s = time.perf_counter() - t0
    ctx = Context(0)
    buf, handles = sst.upload_blocks(ctx, stored)
    in_bytes = sum(len(d) for d, _ in stored)
    t0 = time.perf_counter()
    table = sst.device_table(ctx, buf, handles)  # once per file: murr_sst_block_t[] in HBM
    table_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(args.warmup):
        e = sst.decode(ctx, buf, table)
        del e
    ts, ks = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        e = sst.decode(ctx, buf, table)
        ts.append(time.perf_counter() - t0)
        ks.append(ctx.last_kernel_ms())
        n, kb, vb = e.n, e.key_bytes, e.value_bytes
        del e
    out_bytes = kb + vb + 4 * (n + 1) + 8 * (n + 1) + 9 * n
    med = float(np.median(ts))
    cpu = None if args.no_cpu else sst_cpu_baseline(stored, args.cpu_seconds)
    print(json.dumps({"mode": "sst", "compression": args.sst_compression, "rows": args.rows, "blocks": len(stored),
                      "stored_bytes": in_bytes, "entry_bytes_out": out_bytes, "gen_s": round(gen_s, 1),
                      "block_table_ms_once": round(table_ms, 3),
                      "ms_per_call_median": round(med * 1e3, 3),
                      "entry_decode_kernel_ms": round(float(np.median(ks)), 4),
                      "GB_s_stored_in": round(in_bytes / med / 1e9, 2),
                      "GB_s_in_plus_out": round((in_bytes + out_bytes) / med / 1e9, 2),
                      "entries_per_s": round(n / med, 0), "cpu_baseline": cpu}))


def sst_cpu_baseline(stored, target_s):
    """The oracle's restatement (oracle/murr_sst.c: Snappy/LZ4 + block walk,
    1 thread) over the same stored blocks, repeated for about target_s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    data = np.frombuffer(b"".join(d for d, _ in stored), np.uint8)
    sizes = np.array([len(d) for d, _ in stored], np.int64)
    h = np.stack([np.cumsum(sizes) - sizes, sizes, np.array([c for _, c in stored], np.int64)], axis=1)
    n_entries, reps = 0, 0
    t = time.perf_counter()
    while True:
        n_entries += O.sst_decode_all(data, h)[0]
        reps += 1
        dt = time.perf_counter() - t
        if dt >= target_s:
            break
    return {"value": round(n_entries / dt, 0), "unit": "entries/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{reps} pass(es) over the {len(stored)} stored blocks (inflate + entry decode) in "
                      f"oracle/libmurr_oracle.so oc_sst_decode_all, {dt:.1f} s"}


def visible_gpus():
    """GPUs this process may use, counted without initialising HIP (the rank
    processes do all GPU work): KFD topology nodes with a GPU target, narrowed
    by HIP_/ROCR_/CUDA_VISIBLE_DEVICES.  None when it cannot tell."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(base):
            with open(os.path.join(base, node, "properties")) as f:
                props = dict(ln.split() for ln in f if len(ln.split()) == 2)
            n += int(props.get("gfx_target_version", "0")) != 0
    except (OSError, ValueError):
        return None
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def spawn_ranks(args) -> int:
    """`--gpus N` without WORLD_SIZE: start N rank processes of this script,
    one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set, as torch.distributed.run would), wait for them and return
    the first failing exit code.  This process touches no GPU.  Rank 0 prints
    the JSON line."""
    import signal
    import socket
    import subprocess
    n = args.gpus
    if args.mode != "harness":
        have = visible_gpus()
        if have is not None and have < n:
            print(f"bench: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for pr in list(pending):
            code = pr.poll()
            if code is None:
                continue
            pending.remove(pr)
            if code and not rc:
                rc = code
                for other in pending:  # the others would wait at a barrier for it
                    other.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="B", choices=["A", "B", "C", "D", "E"])
    ap.add_argument("--rows", type=int, default=None, help="rows per block")
    ap.add_argument("--blocks", type=int, default=None, help="blocks per launch")
    ap.add_argument("--mode", default="decode", choices=["decode", "host", "encode", "resident", "sst", "harness"],
                    help="harness: CPU self-test of the multi-rank harness (no GPU, not a measurement)")
    ap.add_argument("--sst-compression", default="snappy", choices=["none", "snappy", "lz4"],
                    help="sst mode: stored block compression")
    ap.add_argument("--keys", type=int, default=1000, help="resident mode: keys per read")
    ap.add_argument("--table-rows", type=int, default=0,
                    help="config D: one table of this many rows split by key range over the ranks "
                         "(configs[3] as written, strong scaling); default: --rows per rank (weak)")
    ap.add_argument("--depth", type=int, default=4, help="host mode: pipeline slots (murr_hstream)")
    ap.add_argument("--host-ring", type=int, default=16, help="host mode: distinct source blocks in the pinned ring")
    ap.add_argument("--ipc", action="store_true", help="resident mode: also time the Arrow IPC message path")
    ap.add_argument("--arena", type=int, default=0,
                    help="decode mode: the K blocks and their outputs as pieces of arenas aligned to this many bytes "
                         "(0: one allocation per buffer)")
    ap.add_argument("--offsets", type=int, default=32, choices=[32, 64],
                    help="row offset width of the decoded blocks (configs A/B/C: u32 row_off32, or u64)")
    ap.add_argument("--resident-stride", type=int, default=0,
                    help="config D: the resident table's utf8 index stride (0: ResidentTable's default)")
    ap.add_argument("--uidx-stride", type=int, default=512,
                    help="decode mode: utf8 index stride of each block (0 = no index)")
    ap.add_argument("--table", default="C", choices=["C", "ref"],
                    help="resident mode: config C table, or the reference read benches' dataset (10 x f32)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the oracle check of the timed output (tuning ablations that skip stores only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--pmc-csv", default=None)
    ap.add_argument("--lanes", type=int, default=None, choices=[1, 2, 3, 4],
                    help="decode: the headline's lanes (tuning A/Bs only; default 1 for every config: the line "
                         "is per launch).  L > 1 = L contexts (streams), so a launch starts on the CUs the "
                         "previous one's tail leaves")
    ap.add_argument("--extra-lanes", type=int, default=3,
                    help="decode: after the one-lane headline, the same steps over this many lanes, every lane's "
                         "last output verified, reported as `lanes` (0 or 1: skip)")
    ap.add_argument("--sync-steps", action="store_true",
                    help="one plan, each step waited for before the next is launched (A/B of the pipelined loop)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the two rocprofv3 --pmc child passes that fill roofline.traffic (N=1)")
    ap.add_argument("--enc-config", default="E", choices=["B", "C", "E"], help="encode mode: column set")
    ap.add_argument("--proj", default=None, help="comma-separated projected columns, or rev (default all, in order)")
    ap.add_argument("--opts", default=None,
                    help="kernel selection (murr_ctx_set_opts), e.g. shape=16x2,lds=163840,mode=local")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    if args.mode != "harness":
        murr_amd.lib()  # raises if the HIP library is not built (no CPU fallback)
    if args.opts:
        set_default_opts(**parse_opts(args.opts))
    if args.rows is None:
        args.rows = {"A": 1000, "B": 100_000, "C": 1_000_000, "D": 1_250_000, "E": 20_000_000}[args.config]
        if args.mode == "encode":
            args.rows = 20_000_000
        if args.mode in ("resident", "sst"):
            args.rows = 1_000_000
    if args.blocks is None:
        args.blocks = {"A": 1, "B": 1000, "C": 1, "D": 1, "E": 1}[args.config]
        if args.mode == "host":
            args.blocks = 200
    if args.mode == "host":
        return run_host(args)
    if args.mode == "encode":
        return run_encode(args)
    if args.mode == "resident":
        return run_resident(args)
    if args.mode == "sst":
        return run_sst(args)
    dist, rank, world, local_rank = dist_init(args)
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    (run_harness if args.mode == "harness" else run_decode)(args, dist, rank, world, local_rank)
    dist.close()


if __name__ == "__main__":
    main()
