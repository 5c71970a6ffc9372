"""Device-resident path: a context (HIP stream + workspace), device buffers, and
the batched decode / encode entry points of the C ABI.

This is the seam the north star measures: blocks of row blobs already in HBM
-> Arrow buffers in HBM (murr_decode_blocks), Arrow buffers in HBM -> row blobs
in HBM (murr_encode_batch).  Buffers are plain device pointers; no torch.
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass

import numpy as np

from . import _abi
from .errors import DeviceError, raise_status
from .schema import DTypeName, SegmentSchema


def device_count() -> int:
    n = C.c_int(0)
    _abi.lib().murr_device_count(C.byref(n))
    return n.value


# murr_opts_t field values by name (murr_codec.h)
KERNELS = {"auto": 0, "jit": 1, "generic": 2}
MODES = {"auto": 0, "local": 1, "split": 2, "cut": 3}
_default_opts: dict = {}
_live = weakref.WeakSet()


def parse_opts(text: str | None) -> dict:
    """"shape=16x2,lds=163840,mode=local" -> set_opts keywords (bench/tools)."""
    out = {}
    for kv in (text or "").split(","):
        if not kv.strip():
            continue
        k, v = kv.split("=", 1)
        k = k.strip()
        if k == "shape":
            nw, r = v.lower().split("x")
            out["shape"] = (int(nw), int(r))
        elif k in ("kernel", "encode_kernel", "mode"):
            out[k] = v
        else:
            out[{"lds": "lds_budget"}.get(k, k)] = int(v)
    return out


def set_default_opts(**kw):
    """Options every live and later Context gets (tests switch kernels with it)."""
    _default_opts.clear()
    _default_opts.update(kw)
    for c in list(_live):
        if c.h:  # (a closed context may linger in the set until collected)
            c.set_opts(**kw)


class Context:
    """murr_ctx_t: one device, one stream, one workspace.  Not thread-safe."""

    def __init__(self, device: int = 0):
        self.L = _abi.lib()
        h = C.c_void_p()
        st = self.L.murr_ctx_create(device, C.byref(h))
        if st:
            raise DeviceError(f"murr_ctx_create(device={device}): {_abi.status_str(st)}")
        self.h = h
        self.device = device
        _live.add(self)
        if _default_opts:
            self.set_opts(**_default_opts)

    def set_opts(self, kernel="auto", mode="auto", shape=None, seg_tiles=0, vrows=0, lds_budget=0, stage=0,
                 encode_kernel="auto", verbose=0, grid=0):
        """murr_ctx_set_opts: kernel selection for this context (all defaults =
        the library's own choice).  kernel / encode_kernel: auto|jit|generic;
        mode: auto|local|split|cut; shape: (waves, chunks) e.g. (5, 3);
        grid: local-mode workgroups (0 auto, -1 one per virtual block)."""
        o = _abi.Opts()
        o.kernel, o.mode, o.encode_kernel = KERNELS[kernel], MODES[mode], KERNELS[encode_kernel]
        o.shape_nw, o.shape_r = shape if shape else (0, 0)
        o.seg_tiles, o.vrows, o.lds_budget, o.stage, o.verbose = seg_tiles, vrows, lds_budget, stage, int(verbose)
        o.grid = grid & 0xFFFFFFFF
        raise_status(self.L.murr_ctx_set_opts(self.h, C.byref(o)), what="murr_ctx_set_opts")
        self.opts_gen = getattr(self, "opts_gen", 0) + 1  # plan caches key on it (no library call per read)

    def opts_key(self) -> tuple:
        """The context's current murr_opts_t as a tuple (plan cache keys)."""
        o = _abi.Opts()
        raise_status(self.L.murr_ctx_get_opts(self.h, C.byref(o)), what="murr_ctx_get_opts")
        return tuple(getattr(o, f) for f, _ in o._fields_)

    def stats(self) -> dict:
        """murr_ctx_stats: decodes, split_retries, last_mode (0 generic, 1 local,
        2 local-cut, 3 split), last_grid, last_shape."""
        s = _abi.CtxStats()
        raise_status(self.L.murr_ctx_stats(self.h, C.byref(s)), what="murr_ctx_stats")
        return {"decodes": s.decodes, "split_retries": s.split_retries,
                "last_mode": ("generic", "local", "cut", "split")[s.last_mode], "last_grid": s.last_grid,
                "last_shape": (s.last_shape_nw, s.last_shape_r), "readback_fallbacks": s.readback_fallbacks,
                "encode_recounts": s.encode_recounts}

    def close(self):
        if self.h:
            self.L.murr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- memory -------------------------------------------------------------
    def alloc(self, nbytes: int) -> "DeviceBuffer":
        p = C.c_void_p()
        raise_status(self.L.murr_dev_alloc(self.h, int(nbytes), C.byref(p)), what="murr_dev_alloc")
        return DeviceBuffer(self, p.value, int(nbytes))

    def upload(self, arr) -> "DeviceBuffer":
        a = np.ascontiguousarray(arr)
        buf = self.alloc(max(a.nbytes, 1))
        if a.nbytes:
            raise_status(self.L.murr_memcpy_h2d(self.h, buf.ptr, a.ctypes.data, a.nbytes), what="h2d")
        return buf

    def sync(self):
        raise_status(self.L.murr_sync(self.h), what="sync")

    def last_kernel(self) -> str:
        """Kernel of the last decode: "murr_jit_decode" or "decode_kernel"."""
        return (self.L.murr_ctx_last_kernel(self.h) or b"").decode()

    def mark(self, which: int):
        """murr_ctx_mark: a timing mark on this context's stream."""
        raise_status(self.L.murr_ctx_mark(self.h, which), what="murr_ctx_mark")

    def mark_ms(self, a: int, b: int, other: "Context | None" = None) -> float:
        """GPU milliseconds from this context's mark a to mark b of `other`
        (default: this context); waits for mark b."""
        o = other or self
        ms = C.c_float()
        raise_status(self.L.murr_ctx_mark_ms(self.h, a, o.h, b, C.byref(ms)), what="murr_ctx_mark_ms")
        return ms.value

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        raise_status(self.L.murr_ctx_last_kernel_ms(self.h, C.byref(ms)), what="kernel time")
        return ms.value


class DeviceBuffer:
    def __init__(self, ctx: Context, ptr: int, nbytes: int):
        self.ctx, self.ptr, self.nbytes = ctx, ptr, nbytes

    def free(self):
        if self.ptr:
            self.ctx.L.murr_dev_free(self.ctx.h, self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            if self.ctx.h:
                self.free()
        except Exception:
            pass

    def download(self, nbytes: int | None = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(max(n, 0), dtype=np.uint8)
        if n:
            raise_status(self.ctx.L.murr_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr + offset, n),
                         what="d2h")
        return out

    def copy_from(self, src: "DeviceBuffer", nbytes: int, dst_offset: int = 0, src_offset: int = 0):
        """Device-to-device copy of nbytes (synchronous)."""
        if nbytes:
            raise_status(self.ctx.L.murr_memcpy_d2d(self.ctx.h, self.ptr + dst_offset, src.ptr + src_offset, nbytes),
                         what="murr_memcpy_d2d")

    def memset(self, value: int = 0):
        raise_status(self.ctx.L.murr_memset_dev(self.ctx.h, self.ptr, value, self.nbytes), what="memset")


@dataclass
class DeviceBlock:
    """murr_block_t: row blobs back to back + row offsets (n_rows + 1), and
    optionally its utf8 index (murr_utf8_index, built by `index_utf8`).
    Offsets are u64 (`row_off`) or u32 (`row_off32`, which the decode then
    reads instead: half the index bytes; `narrow` makes them)."""
    data: DeviceBuffer
    row_off: "DeviceBuffer | None"
    n_rows: int
    data_bytes: int
    uidx: "DeviceBuffer | None" = None
    stride: int = 0
    row_off32: "DeviceBuffer | None" = None

    @property
    def offset_width(self) -> int:
        return 4 if self.row_off32 is not None else 8

    def c_block(self, cb=None):
        """The murr_block_t of this block (filled into `cb` when given)."""
        cb = cb if cb is not None else _abi.Block()
        cb.data = self.data.ptr
        cb.row_off = self.row_off.ptr if self.row_off is not None else None
        cb.n_rows, cb.data_bytes = self.n_rows, self.data_bytes
        cb.row_off32 = self.row_off32.ptr if self.row_off32 is not None else None
        return cb

    def narrow(self, ctx: "Context", keep64: bool = False) -> "DeviceBlock":
        """The same block with u32 row offsets (murr_row_off_narrow; raises
        when the block's bytes reach 2^32).  keep64: keep the u64 ones too."""
        if self.row_off32 is not None:
            return self
        buf = ctx.alloc(4 * (self.n_rows + 1))
        raise_status(ctx.L.murr_row_off_narrow(ctx.h, self.row_off.ptr, self.n_rows, buf.ptr),
                     what="murr_row_off_narrow")
        return DeviceBlock(self.data, self.row_off if keep64 else None, self.n_rows, self.data_bytes, self.uidx,
                           self.stride, buf)

    def host_offsets(self) -> np.ndarray:
        """The row offsets as host u64 (either width on the device)."""
        if self.row_off32 is not None:
            return self.row_off32.download(4 * (self.n_rows + 1)).view(np.uint32).astype(np.uint64)
        return self.row_off.download(8 * (self.n_rows + 1)).view(np.uint64).copy()

    def index_utf8(self, ctx: "Context", segment: SegmentSchema, stride: int = 512) -> "DeviceBlock":
        """Build the block's utf8 index (per `stride` rows, every utf8 column's
        string bytes before it): lets one large block be decoded by the whole
        GPU in one pass.  A layout without utf8 columns needs none."""
        n = int(ctx.L.murr_utf8_index_len(C.byref(segment.c), self.n_rows, stride))
        if n == 0:
            self.uidx, self.stride = None, 0
            return self
        buf = ctx.alloc(8 * n)
        cb = self.c_block()
        raise_status(ctx.L.murr_utf8_index(ctx.h, C.byref(segment.c), C.byref(cb), stride, buf.ptr),
                     what="murr_utf8_index")
        self.uidx, self.stride = buf, stride
        return self

    @classmethod
    def upload(cls, ctx: Context, data: np.ndarray, row_off: np.ndarray, width: int = 8) -> "DeviceBlock":
        """A block from host bytes; width 4 uploads the offsets as u32."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if width == 4:
            ro = np.ascontiguousarray(row_off, dtype=np.uint64)
            if ro.size and int(ro[-1]) >= 1 << 32:
                raise ValueError("u32 row offsets: the block's bytes reach 2^32")
            return cls(ctx.upload(data), None, ro.size - 1, data.nbytes, row_off32=ctx.upload(ro.astype(np.uint32)))
        row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
        return cls(ctx.upload(data), ctx.upload(row_off), row_off.size - 1, data.nbytes)


class DecodeOutputs:
    """Device output buffers for nblocks x nproj Arrow arrays (murr_array_t)."""

    def __init__(self, ctx: Context, segment: SegmentSchema, proj, blocks):
        self.ctx = ctx
        self.proj = list(proj)
        self.blocks = blocks
        np_ = len(self.proj)
        self.arrays = (_abi.Array * max(len(blocks) * np_, 1))()
        self.bufs = []
        L = ctx.L
        fixed = segment.bitset_size + segment.capacity
        for b, blk in enumerate(blocks):
            n = blk.n_rows
            bm = int(L.murr_bitmap_bytes(n))
            utf8_cap = max(blk.data_bytes - 0, 0)  # strings are a subset of the blob bytes
            for p, ci in enumerate(self.proj):
                col = segment.columns[ci]
                a = self.arrays[b * np_ + p]
                if col.dtype == DTypeName.Utf8:
                    vb = max(utf8_cap, 8)
                    offs = ctx.alloc((n + 1) * 4)
                    self.bufs.append(offs)
                    a.offsets = offs.ptr
                    a.values_cap = vb
                elif col.dtype == DTypeName.Bool:
                    vb = bm
                else:
                    vb = n * col.dtype.size()
                vals = ctx.alloc(max(vb, 8))
                valid = ctx.alloc(max(bm, 8))
                self.bufs += [vals, valid]
                a.values = vals.ptr
                a.validity = valid.ptr
        del fixed

    def array(self, b: int, p: int):
        return self.arrays[b * len(self.proj) + p]


def decode_blocks(ctx: Context, segment: SegmentSchema, proj, blocks, outs: DecodeOutputs | None = None):
    """murr_decode_blocks over device-resident blocks.  Returns the outputs
    object (null counts / data lengths filled)."""
    proj = list(proj)
    outs = outs or DecodeOutputs(ctx, segment, proj, blocks)
    cb = (_abi.Block * max(len(blocks), 1))()
    for i, blk in enumerate(blocks):
        blk.c_block(cb[i])
    pj = (C.c_uint32 * max(len(proj), 1))(*proj)
    err = _abi.Error()
    ix = [b.uidx for b in blocks]
    if any(u is not None for u in ix):
        strides = {b.stride for b in blocks if b.uidx is not None}
        if len(strides) != 1:
            raise ValueError("blocks of one decode share one utf8 index stride")
        up = (C.c_void_p * len(blocks))(*[u.ptr if u is not None else None for u in ix])
        st = ctx.L.murr_decode_blocks_ix(ctx.h, C.byref(segment.c), pj, len(proj), cb, len(blocks), up,
                                         strides.pop(), outs.arrays, C.byref(err))
    else:
        st = ctx.L.murr_decode_blocks(ctx.h, C.byref(segment.c), pj, len(proj), cb, len(blocks),
                                      outs.arrays, C.byref(err))
    raise_status(st, err, "murr_decode_blocks")
    return outs


class DecodePlan:
    """murr_decode_plan: one decode over fixed blocks and output buffers,
    prepared once (shape, descriptors, kernel arguments uploaded); run()
    repeats it with one launch and one small read-back (murr_decode_run).
    The blocks and `outs` must stay alive and in place while the plan lives."""

    def __init__(self, ctx: Context, segment: SegmentSchema, proj, blocks, outs: "DecodeOutputs | None" = None):
        self.ctx, self.segment, self.proj, self.blocks = ctx, segment, list(proj), list(blocks)
        self.outs = outs or DecodeOutputs(ctx, segment, self.proj, self.blocks)
        k = max(len(self.blocks), 1)
        self._cb = (_abi.Block * k)()
        for i, blk in enumerate(self.blocks):
            blk.c_block(self._cb[i])
        self._pj = (C.c_uint32 * max(len(self.proj), 1))(*self.proj)
        ix = [b.uidx for b in self.blocks]
        self._ux, stride = None, 0
        if any(u is not None for u in ix):
            strides = {b.stride for b in self.blocks if b.uidx is not None}
            if len(strides) != 1:
                raise ValueError("blocks of one decode share one utf8 index stride")
            stride = strides.pop()
            self._ux = (C.c_void_p * k)(*[u.ptr if u is not None else None for u in ix])
        h = C.c_void_p()
        st = ctx.L.murr_decode_plan(ctx.h, C.byref(segment.c), self._pj, len(self.proj), self._cb, len(self.blocks),
                                    self._ux, stride, self.outs.arrays, C.byref(h))
        raise_status(st, what="murr_decode_plan")
        self.h = h.value
        self._err = _abi.Error()

    def time_every(self, every: int):
        """murr_plan_time_every: time one run in `every` (0: none)."""
        raise_status(self.ctx.L.murr_plan_time_every(self.h, every), what="murr_plan_time_every")

    def run(self) -> "DecodeOutputs":
        st = self.ctx.L.murr_decode_run(self.h, C.byref(self._err))
        raise_status(st, self._err, "murr_decode_run")
        return self.outs

    def run_async(self):
        """Launch a run and return (murr_decode_run_async); wait() finishes it."""
        if not self.h:
            raise ValueError("DecodePlan is closed")
        raise_status(self.ctx.L.murr_decode_run_async(self.h), what="murr_decode_run_async")
        self._inflight, self._drained = True, None

    def wait(self) -> "DecodeOutputs":
        if not self.h:
            # closed with a run in flight (a plan cache evicted it): close()
            # finished that run; hand over its result once
            d, self._drained = getattr(self, "_drained", None), None
            if d is None:
                raise ValueError("DecodePlan is closed and has no run to wait for")
            if isinstance(d, BaseException):
                raise d
            return d
        self._inflight = False
        st = self.ctx.L.murr_decode_run_wait(self.h, C.byref(self._err))
        raise_status(st, self._err, "murr_decode_run_wait")
        return self.outs

    @property
    def inflight(self) -> bool:
        return bool(getattr(self, "_inflight", False))

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:
            if self.inflight:  # never free a plan under its own running launch
                try:
                    self._drained = self.wait()
                except Exception as e:  # kept for the caller's wait()
                    self._drained = e
            self.ctx.L.murr_plan_free(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def download_array(ctx: Context, a, dtype: int, n: int) -> dict:
    """Copy one decoded Arrow array (murr_array_t) back to host buffers."""
    def d2h(ptr, nbytes):
        out = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            raise_status(ctx.L.murr_memcpy_d2h(ctx.h, out.ctypes.data, ptr, nbytes), what="d2h")
        return out
    bm = int(ctx.L.murr_bitmap_bytes(n))
    res = {"dtype": dtype, "length": n, "null_count": a.null_count,
           "validity": d2h(a.validity, bm).tobytes() if a.null_count else None,
           "validity_raw": d2h(a.validity, bm).tobytes() if n else b"",
           "offsets": None}
    if dtype == int(DTypeName.Utf8):
        res["offsets"] = d2h(a.offsets, (n + 1) * 4).view(np.int32)
        res["values"] = d2h(a.values, a.data_len).tobytes()
    elif dtype == int(DTypeName.Bool):
        res["values"] = d2h(a.values, bm).tobytes()
    else:
        res["values"] = d2h(a.values, a.data_len).tobytes()
    return res


def encode_block(ctx: Context, segment: SegmentSchema, cols, n: int, stride: int = 512) -> "DeviceBlock":
    """murr_encode_batch_ix: Arrow columns (device) -> a decode block with its
    utf8 index (a layout without utf8 columns gets none)."""
    cin, ub = _col_in(cols)
    blob_cap = int(ctx.L.murr_encode_bound(C.byref(segment.c), n, ub))
    blob = ctx.alloc(max(blob_cap, 16))
    row_off = ctx.alloc((n + 1) * 8)
    nix = int(ctx.L.murr_utf8_index_len(C.byref(segment.c), n, stride))
    uidx = ctx.alloc(8 * nix) if nix else None
    blen = C.c_uint64()
    err = _abi.Error()
    st = ctx.L.murr_encode_batch_ix(ctx.h, C.byref(segment.c), cin, n, blob.ptr, blob_cap, row_off.ptr, stride,
                                    uidx.ptr if uidx is not None else None, C.byref(blen), C.byref(err))
    raise_status(st, err, "murr_encode_batch_ix")
    return DeviceBlock(blob, row_off, n, blen.value, uidx, stride if uidx is not None else 0)


def _col_in(cols):
    cin = (_abi.ColIn * max(len(cols), 1))()
    ub = (C.c_uint64 * max(len(cols), 1))()
    for i, c in enumerate(cols):
        cin[i].values = c["values"].ptr if c.get("values") is not None else None
        cin[i].validity = c["validity"].ptr if c.get("validity") is not None else None
        cin[i].offsets = c["offsets"].ptr if c.get("offsets") is not None else None
        cin[i].offset = int(c.get("offset", 0))
        ub[i] = int(c.get("utf8_bytes", 0))
    return cin, ub


def encode_batch(ctx: Context, segment: SegmentSchema, cols, n: int, blob_cap: int | None = None, out=None):
    """murr_encode_batch over device-resident Arrow columns.

    cols: per segment column dict {values: DeviceBuffer, validity: DeviceBuffer|None,
    offsets: DeviceBuffer|None, offset: int, utf8_bytes: int}.
    out: optional (blob, row_off) DeviceBuffers to write into (a repeated
    encode of the same shape reuses them instead of allocating each call).
    Returns (blob DeviceBuffer, row_off DeviceBuffer, blob_len)."""
    cin, ub = _col_in(cols)
    if blob_cap is None:
        blob_cap = int(ctx.L.murr_encode_bound(C.byref(segment.c), n, ub))
    if out is not None:
        blob, row_off = out
        if blob.nbytes < max(blob_cap, 16) or row_off.nbytes < (n + 1) * 8:
            raise ValueError("encode_batch: out buffers smaller than the encode bound")
    else:
        blob = ctx.alloc(max(blob_cap, 16))
        row_off = ctx.alloc((n + 1) * 8)
    blen = C.c_uint64()
    err = _abi.Error()
    st = ctx.L.murr_encode_batch(ctx.h, C.byref(segment.c), cin, n, blob.ptr, blob_cap, row_off.ptr,
                                 C.byref(blen), C.byref(err))
    raise_status(st, err, "murr_encode_batch")
    return blob, row_off, blen.value
