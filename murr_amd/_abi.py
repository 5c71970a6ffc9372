"""ctypes binding of include/murr_codec.h (libmurr_codec.so, built in-tree).

Loading fails loudly: there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# MURR_LIB: load another build of the same library (the tuning build of
# tools/); announced on stderr whenever it is set, so no run swaps it in silently
ABI_VERSION = 2  # include/murr_codec.h MURR_ABI_VERSION
LIB_PATH = os.environ.get("MURR_LIB") or os.path.join(HERE, "libmurr_codec.so")
HEADER = os.path.join(ROOT, "include", "murr_codec.h")
PLAN_TIME_EVERY = 4  # MURR_PLAN_TIME_EVERY: a prepared plan times one run in this many

# murr_status_t
OK, E_INVALID_UTF8, E_DTYPE, E_BAD_COLUMN, E_OFFSET_OVERFLOW, E_MALFORMED_ROW, E_CAPACITY, \
    E_ARGUMENT, E_NULL_KEY, E_HIP, E_INTERNAL, E_ARROW, E_NO_DEVICE = range(13)


class Column(C.Structure):
    _fields_ = [("index", C.c_uint32), ("dtype", C.c_uint32), ("offset", C.c_uint32),
                ("size", C.c_uint32)]


class Segment(C.Structure):
    _fields_ = [("ncols", C.c_uint32), ("bitset_size", C.c_uint32), ("capacity", C.c_uint32),
                ("_pad", C.c_uint32), ("cols", C.POINTER(Column))]


class Error(C.Structure):
    _fields_ = [("status", C.c_int32), ("hip_error", C.c_int32), ("block", C.c_uint32),
                ("column", C.c_uint32), ("row", C.c_uint64), ("required", C.c_uint64)]


class Opts(C.Structure):
    """murr_opts_t: kernel selection of one context (tests, benchmarks)."""
    _fields_ = [(n, C.c_uint32) for n in ("kernel", "mode", "shape_nw", "shape_r", "seg_tiles", "vrows",
                                          "lds_budget", "stage", "encode_kernel", "verbose", "grid",
                                          "reserved")]


class CtxStats(C.Structure):
    _fields_ = [("decodes", C.c_uint64), ("split_retries", C.c_uint64), ("last_mode", C.c_uint32),
                ("last_grid", C.c_uint32), ("last_shape_nw", C.c_uint32), ("last_shape_r", C.c_uint32),
                ("readback_fallbacks", C.c_uint64), ("encode_recounts", C.c_uint64)]


class Block(C.Structure):
    """murr_block_t: row_off (u64), or row_off32 (u32) when set."""
    _fields_ = [("data", C.c_void_p), ("row_off", C.c_void_p), ("n_rows", C.c_uint64),
                ("data_bytes", C.c_uint64), ("row_off32", C.c_void_p)]


class ArrowSchema(C.Structure):
    """struct ArrowSchema (Arrow C Data Interface, include/murr_codec.h)."""
    _fields_ = [("format", C.c_char_p), ("name", C.c_char_p), ("metadata", C.c_char_p), ("flags", C.c_int64),
                ("n_children", C.c_int64), ("children", C.c_void_p), ("dictionary", C.c_void_p),
                ("release", C.c_void_p), ("private_data", C.c_void_p)]


class ArrowArray(C.Structure):
    """struct ArrowArray (Arrow C Data Interface, include/murr_codec.h)."""
    _fields_ = [("length", C.c_int64), ("null_count", C.c_int64), ("offset", C.c_int64), ("n_buffers", C.c_int64),
                ("n_children", C.c_int64), ("buffers", C.c_void_p), ("children", C.c_void_p),
                ("dictionary", C.c_void_p), ("release", C.c_void_p), ("private_data", C.c_void_p)]


class Array(C.Structure):
    _fields_ = [("values", C.c_void_p), ("validity", C.c_void_p), ("offsets", C.c_void_p),
                ("values_cap", C.c_uint64), ("null_count", C.c_uint64), ("data_len", C.c_uint64)]


class ColIn(C.Structure):
    _fields_ = [("values", C.c_void_p), ("validity", C.c_void_p), ("offsets", C.c_void_p),
                ("offset", C.c_uint64)]


class ShardRead(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("index", C.c_void_p), ("arena", C.c_void_p), ("row_off", C.c_void_p),
                ("q_end", C.c_uint64)]


class SstBlock(C.Structure):
    _fields_ = [("data", C.c_void_p), ("size", C.c_uint64), ("compression", C.c_uint32), ("_pad", C.c_uint32)]


class SstResult(C.Structure):
    _fields_ = [("n", C.c_uint64), ("keys", C.c_void_p), ("key_offsets", C.c_void_p), ("values", C.c_void_p),
                ("value_offsets", C.c_void_p), ("seqs", C.c_void_p), ("types", C.c_void_p),
                ("key_bytes", C.c_uint64), ("value_bytes", C.c_uint64)]


class HostArray(C.Structure):
    _fields_ = [("values", C.c_void_p), ("validity", C.c_void_p), ("offsets", C.c_void_p),
                ("length", C.c_uint64), ("null_count", C.c_uint64), ("values_len", C.c_uint64),
                ("dtype", C.c_uint32), ("_pad", C.c_uint32)]


class HStreamStats(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("h2d_ms", C.c_double), ("kernel_ms", C.c_double), ("d2h_ms", C.c_double),
                ("h2d_bytes", C.c_uint64), ("d2h_bytes", C.c_uint64), ("timed_batches", C.c_uint64),
                ("host_submit_ms", C.c_double), ("host_next_ms", C.c_double),
                ("host_wait_ms", C.c_double)]


class HostColIn(C.Structure):
    _fields_ = [("col", ColIn), ("values_bytes", C.c_uint64)]


P = C.c_void_p
PP = C.POINTER(C.c_void_p)
U32, U64, I32 = C.c_uint32, C.c_uint64, C.c_int

# name -> (restype, argtypes); mirrors include/murr_codec.h one to one.
SIGNATURES = {
    "murr_abi_version": (U32, []),
    "murr_arrow_export": (I32, [C.POINTER(HostArray), U32, C.POINTER(C.c_char_p), P, P]),
    "murr_dtype_size": (I32, [U32]),
    "murr_segment_init": (I32, [C.POINTER(U32), U32, C.POINTER(Column), C.POINTER(Segment)]),
    "murr_segment_prepare": (I32, [P, C.POINTER(Segment)]),
    "murr_bitmap_bytes": (U64, [U64]),
    "murr_ctx_create": (I32, [I32, PP]),
    "murr_ctx_destroy": (None, [P]),
    "murr_ctx_stream": (P, [P]),
    "murr_ctx_last_kernel_ms": (I32, [P, C.POINTER(C.c_float)]),
    "murr_ctx_last_kernel": (C.c_char_p, [P]),
    "murr_device_count": (I32, [C.POINTER(I32)]),
    "murr_ctx_set_opts": (I32, [P, C.POINTER(Opts)]),
    "murr_ctx_get_opts": (I32, [P, C.POINTER(Opts)]),
    "murr_ctx_stats": (I32, [P, C.POINTER(CtxStats)]),
    "murr_jit_cache_limit": (I32, [U32, C.POINTER(U32), C.POINTER(U32)]),
    "murr_dev_alloc": (I32, [P, U64, PP]),
    "murr_dev_free": (I32, [P, P]),
    "murr_host_alloc": (I32, [P, U64, PP]),
    "murr_host_free": (I32, [P, P]),
    "murr_memcpy_h2d": (I32, [P, P, P, U64]),
    "murr_memcpy_d2h": (I32, [P, P, P, U64]),
    "murr_memcpy_d2d": (I32, [P, P, P, U64]),
    "murr_memcpy_peer": (I32, [P, P, P, I32, U64]),
    "murr_row_off_narrow": (I32, [P, P, U64, P]),
    "murr_shard_of": (I32, [P, P, U64, U64, U32, P]),
    "murr_memset_dev": (I32, [P, P, I32, U64]),
    "murr_sync": (I32, [P]),
    "murr_decode_blocks": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Block), U32,
                                 C.POINTER(Array), C.POINTER(Error)]),
    "murr_decode_enqueue": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Block), U32,
                                  C.POINTER(Array)]),
    "murr_decode_wait": (I32, [P, C.POINTER(Error)]),
    "murr_decode_blocks_ix": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Block), U32,
                                    C.POINTER(C.c_void_p), U32, C.POINTER(Array), C.POINTER(Error)]),
    "murr_decode_enqueue_ix": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Block), U32,
                                     C.POINTER(C.c_void_p), U32, C.POINTER(Array)]),
    "murr_utf8_index_len": (U64, [C.POINTER(Segment), U64, U32]),
    "murr_decode_plan": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Block), U32,
                               C.POINTER(C.c_void_p), U32, C.POINTER(Array), PP]),
    "murr_decode_run": (I32, [P, C.POINTER(Error)]),
    "murr_decode_run_async": (I32, [P]),
    "murr_decode_run_wait": (I32, [P, C.POINTER(Error)]),
    "murr_plan_free": (None, [P]),
    "murr_plan_time_every": (I32, [P, U32]),
    "murr_ctx_mark": (I32, [P, U32]),
    "murr_ctx_mark_ms": (I32, [P, U32, P, U32, C.POINTER(C.c_float)]),
    "murr_sst_decode": (I32, [P, C.POINTER(SstBlock), U32, C.POINTER(SstResult), C.POINTER(Error)]),
    "murr_sst_result_free": (None, [P, C.POINTER(SstResult)]),
    "murr_utf8_index": (I32, [P, C.POINTER(Segment), C.POINTER(Block), U32, P]),
    "murr_utf8_index_update": (I32, [P, C.POINTER(Segment), C.POINTER(Block), U64, U32, P]),
    "murr_utf8_row_lengths": (I32, [P, C.POINTER(Segment), C.POINTER(Block), U64, P]),
    "murr_index_cache_rows": (I32, [P, P, P, P, U32, C.POINTER(Error)]),
    "murr_encode_batch_ix": (I32, [P, C.POINTER(Segment), C.POINTER(ColIn), U64, P, U64, P, U32, P,
                                   C.POINTER(U64), C.POINTER(Error)]),
    "murr_encode_bound": (U64, [C.POINTER(Segment), U64, C.POINTER(U64)]),
    "murr_encode_batch": (I32, [P, C.POINTER(Segment), C.POINTER(ColIn), U64, P, U64, P,
                                C.POINTER(U64), C.POINTER(Error)]),
    "murr_encode_batch_at": (I32, [P, C.POINTER(Segment), C.POINTER(ColIn), U64, P, U64, P, U64,
                                   C.POINTER(U64), C.POINTER(Error)]),
    "murr_builder_new": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, U64, PP]),
    "murr_builder_add_row": (I32, [P, P, U64]),
    "murr_builder_add_empty": (I32, [P]),
    "murr_builder_add_rows": (I32, [P, C.POINTER(C.c_void_p), C.POINTER(U64), U64]),
    "murr_builder_build": (I32, [P, C.POINTER(HostArray), C.POINTER(Error)]),
    "murr_builder_last_timing": (I32, [P, C.POINTER(C.c_double), C.POINTER(C.c_float),
                                       C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "murr_builder_free": (None, [P]),
    "murr_hstream_new": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, U32, PP]),
    "murr_hstream_submit": (I32, [P, P, P, U64, U32, C.POINTER(Error)]),
    "murr_hstream_submit32": (I32, [P, P, P, U64, U32, C.POINTER(Error)]),
    "murr_hstream_next": (I32, [P, C.POINTER(HostArray), C.POINTER(Error)]),
    "murr_hstream_stats": (I32, [P, C.POINTER(HStreamStats)]),
    "murr_hstream_free": (None, [P]),
    "murr_reader_new": (I32, [P, C.POINTER(Segment), PP]),
    "murr_reader_read": (I32, [P, P, P, P, U64, U64, P, P, U64, U64, C.POINTER(U32), U32,
                               C.POINTER(HostArray), C.POINTER(Error)]),
    "murr_reader_free": (None, [P]),
    "murr_read_plan_new": (I32, [P, C.POINTER(Segment), P, P, P, P, U64, U64, C.POINTER(U32), U32, U64, PP]),
    "murr_read_plan_run_device": (I32, [P, P, P, U64, C.POINTER(Array), C.POINTER(Error)]),
    "murr_read_plan_run": (I32, [P, P, P, U64, U64, C.POINTER(HostArray), C.POINTER(Error)]),
    "murr_read_plan_capacity": (U64, [P]),
    "murr_read_plan_free": (None, [P]),
    "murr_encode_host": (I32, [P, C.POINTER(Segment), C.POINTER(HostColIn), U64,
                               C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(U64),
                               C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(Error)]),
    "murr_index_build": (I32, [P, P, P, U64, U64, PP, C.POINTER(Error)]),
    "murr_index_free": (None, [P]),
    "murr_index_append": (I32, [P, P, P, P, U64, U64, C.POINTER(Error)]),
    "murr_index_info": (I32, [P, C.POINTER(U64), C.POINTER(U64)]),
    "murr_index_prefer_seq": (I32, [P, P, P, C.POINTER(Error)]),
    "murr_multi_gather": (I32, [P, C.POINTER(ShardRead), U32, P, P, P, U64, P, P, P, U64, P, C.POINTER(Error)]),
    "murr_multi_gather_copy": (I32, [P, C.POINTER(ShardRead), U32, P, U64, P, P, P, C.POINTER(Error)]),
    "murr_index_lookup": (I32, [P, P, P, P, U64, P]),
    "murr_index_gather": (I32, [P, P, P, P, U64, P, P, P, U64, P, P, P]),
    "murr_index_gather_copy": (I32, [P, P, U64, P, P, P, P]),
    "murr_ipc_schema": (I32, [C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(C.c_char_p), U32, P, U64,
                              C.POINTER(U64)]),
    "murr_ipc_batch_host": (I32, [C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(HostArray), U64, U32, P,
                                  U64, C.POINTER(U64)]),
    "murr_ipc_batch_device": (I32, [P, C.POINTER(Segment), C.POINTER(U32), U32, C.POINTER(Array), U64, U32, P,
                                    U64, C.POINTER(U64), C.POINTER(Error)]),
    "murr_ipc_eos": (U64, [P]),
    "murr_status_str": (C.c_char_p, [I32]),
}

_lib = None


def header_symbols():
    """Every function the public header declares."""
    with open(HEADER) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(murr_[a-z0-9_]+)\s*\(", src)))


def lib():
    """Load libmurr_codec.so; raises if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libmurr_codec.so not built at {LIB_PATH}; run "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        if os.environ.get("MURR_LIB"):
            import sys
            print(f"murr_amd: MURR_LIB set, loading {LIB_PATH} instead of the in-tree release library",
                  file=sys.stderr)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        got = L.murr_abi_version()
        if got != ABI_VERSION:  # descriptor strides differ: never pass arrays across versions
            raise ImportError(f"{LIB_PATH}: ABI version {got}, this binding expects {ABI_VERSION}")
        _lib = L
    return _lib


def status_str(st: int) -> str:
    return lib().murr_status_str(st).decode()
