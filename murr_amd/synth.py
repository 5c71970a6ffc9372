"""Synthetic workloads of BASELINE.json's configs, as Arrow column buffers (numpy).

Shapes follow the reference's bench data (benches/common/data.rs:24-68,
benches/common/dataset.rs:24-55: `col_i = i as f32`, key `i.to_string()`) and
SURVEY.md §8(d):
  A  {key, v: f32 = i}                                  (read_plain CPU case)
  B  {key, f: f32 = i, s: utf8 = i.to_string()}          (read_block shape)
  C  16 mixed nullable columns, 10 % nulls (seed 42), uniform values (seed 43)
  D  config C schema, sharded by key range
  E  {key, col_0..col_9: f32 = i}                       (write shape)
Seeds are numpy PCG64 (not rand's StdRng); the reference's exact key samples are
not reproducible without Rust and do not matter for a codec.
"""
from __future__ import annotations

import numpy as np
import pyarrow as pa

from .schema import DTypeName

D = DTypeName
CONFIG_C_DTYPES = [D.Bool, D.Int8, D.Int16, D.Int32, D.Int64, D.UInt8, D.UInt16, D.UInt32, D.UInt64,
                   D.Float32, D.Float64, D.Utf8, D.Utf8, D.Float32, D.Float64, D.Int64]
_NP = {D.Int8: np.int8, D.Int16: np.int16, D.Int32: np.int32, D.Int64: np.int64, D.UInt8: np.uint8,
       D.UInt16: np.uint16, D.UInt32: np.uint32, D.UInt64: np.uint64, D.Float32: np.float32,
       D.Float64: np.float64}


def pack_bits(mask: np.ndarray) -> np.ndarray:
    """LSB-first Arrow bitmap of a bool array."""
    return np.packbits(np.asarray(mask, dtype=bool), bitorder="little")


def int_strings(start: int, n: int):
    """`i.to_string()` for i in [start, start+n): (offsets int32, data uint8).
    Vectorised: the numbers with the same digit count form contiguous runs,
    each written as a [run, width] digit matrix, so 1e8 keys take seconds."""
    offs = np.zeros(n + 1, dtype=np.int64)
    parts = []
    i, at = start, 0
    while i < start + n:
        width = len(str(i))
        hi = min(start + n, 10 ** width)  # numbers below 10**width have `width` digits
        v = np.arange(i, hi, dtype=np.int64)
        m = v.size
        digits = np.empty((m, width), dtype=np.uint8)
        for j in range(width):
            digits[:, j] = (v // 10 ** (width - 1 - j)) % 10 + 48
        parts.append(digits.ravel())
        offs[at + 1:at + m + 1] = offs[at] + width * np.arange(1, m + 1, dtype=np.int64)
        i, at = hi, at + m
    data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return offs.astype(np.int32), data


def random_ascii(rng, n: int, max_len: int = 32):
    lens = rng.integers(0, max_len + 1, size=n)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0x20, 0x7F, size=int(offs[-1]), dtype=np.uint8)
    return offs.astype(np.int32), data


def column(dtype, values=None, valid=None, offsets=None, data=None, n=None):
    """Arrow column as buffers; null slots of fixed columns are left as given."""
    dtype = DTypeName(dtype)
    n = n if n is not None else (len(offsets) - 1 if offsets is not None else len(values))
    c = {"dtype": dtype, "n": n, "validity": None, "offsets": None, "offset": 0}
    if valid is not None and not np.all(valid):
        c["validity"] = pack_bits(valid)
    if dtype == D.Utf8:
        c["offsets"] = np.ascontiguousarray(offsets, dtype=np.int32)
        c["values"] = np.ascontiguousarray(data, dtype=np.uint8)
        if c["values"].size == 0:
            c["values"] = np.zeros(16, dtype=np.uint8)
    elif dtype == D.Bool:
        c["values"] = pack_bits(values)
    else:
        c["values"] = np.ascontiguousarray(values, dtype=_NP[dtype])
    return c


def to_arrow(c) -> pa.Array:
    dt = c["dtype"]
    n = c["n"]
    valid = pa.py_buffer(c["validity"].tobytes()) if c["validity"] is not None else None
    if dt == D.Utf8:
        return pa.Array.from_buffers(pa.string(), n, [valid, pa.py_buffer(c["offsets"].tobytes()),
                                                     pa.py_buffer(c["values"].tobytes())])
    return pa.Array.from_buffers(dt.arrow_dtype(), n, [valid, pa.py_buffer(c["values"].tobytes())])


def config_a(n: int = 1000, start: int = 0):
    """configs[0], benches/read_plain.rs on CPU at its plumbing size: one
    FLOAT32 column, f = i, no nulls."""
    return [column(D.Float32, np.arange(start, start + n).astype(np.float32))]


def config_b(n: int, start: int = 0, null_frac: float = 0.0, seed: int = 42):
    """{f: f32 = i, s: utf8 = i.to_string()} (key column omitted: not in the blob)."""
    i = np.arange(start, start + n)
    offs, data = int_strings(start, n)
    valid_f = valid_s = None
    if null_frac:
        rng = np.random.default_rng(seed)
        valid_f = rng.random(n) >= null_frac
        valid_s = rng.random(n) >= null_frac
        offs, data = _null_strings(offs, data, valid_s)
    return [column(D.Float32, i.astype(np.float32) * (valid_f if valid_f is not None else 1), valid_f),
            column(D.Utf8, valid=valid_s, offsets=offs, data=data)]


def _null_strings(offs, data, valid):
    """Drop the bytes of null strings (Arrow null -> empty slot, repeated offset)."""
    lens = np.diff(offs.astype(np.int64)) * valid
    keep = np.repeat(valid, np.diff(offs.astype(np.int64)))
    noffs = np.zeros(len(offs), dtype=np.int64)
    np.cumsum(lens, out=noffs[1:])
    return noffs.astype(np.int32), data[keep]


def config_c(n: int, start: int = 0, null_frac: float = 0.10, seed_nulls: int = 42,
             seed_vals: int = 43):
    """16 mixed nullable columns."""
    rn = np.random.default_rng(seed_nulls + start)
    rv = np.random.default_rng(seed_vals + start)
    cols = []
    for j, dt in enumerate(CONFIG_C_DTYPES):
        valid = rn.random(n) >= null_frac
        if dt == D.Utf8:
            offs, data = int_strings(start, n) if j == 11 else random_ascii(rv, n)
            offs, data = _null_strings(offs, data, valid)
            cols.append(column(dt, valid=valid, offsets=offs, data=data))
        elif dt == D.Bool:
            cols.append(column(dt, rv.random(n) < 0.5, valid))
        elif dt in (D.Float32, D.Float64):
            v = (rv.standard_normal(n) * 1e6).astype(_NP[dt])
            cols.append(column(dt, np.where(valid, v, 0).astype(_NP[dt]), valid))
        else:
            info = np.iinfo(_NP[dt])
            v = rv.integers(info.min, info.max, size=n, dtype=_NP[dt], endpoint=True)
            cols.append(column(dt, np.where(valid, v, 0).astype(_NP[dt]), valid))
    return cols


def config_e(n: int, ncols: int = 10, start: int = 0):
    """{col_0..col_{ncols-1}: f32 = i} (benches/write.rs:21-22, data.rs:54-56)."""
    v = np.arange(start, start + n, dtype=np.int64).astype(np.float32)  # `i as f32`
    return [column(D.Float32, v) for _ in range(ncols)]


def ref_batch(start: int, n: int, ncols: int = 10) -> pa.RecordBatch:
    """Rows [start, start+n) of the reference benches' dataset
    (benches/common/dataset.rs:24-55): key = i.to_string(), col_j = i as f32."""
    ko, kd = int_strings(start, n)
    keys = pa.Array.from_buffers(pa.string(), n, [None, pa.py_buffer(ko), pa.py_buffer(kd)])
    v = pa.array(np.arange(start, start + n, dtype=np.int64).astype(np.float32))
    return pa.RecordBatch.from_arrays([keys] + [v] * ncols, names=["key"] + [f"col_{j}" for j in range(ncols)])


def ref_schema(ncols: int = 10):
    from .schema import ColumnSchema, TableSchema
    cols = {"key": ColumnSchema(D.Utf8, False)}
    cols.update({f"col_{j}": ColumnSchema(D.Float32) for j in range(ncols)})
    return TableSchema("key", cols)


def utf8_bytes(cols):
    """Per column string bytes (for murr_encode_bound)."""
    return [int(c["offsets"][-1] - c["offsets"][0]) if c["dtype"] == D.Utf8 else 0 for c in cols]


def upload_columns(ctx, cols):
    """Arrow buffers -> device buffers (dicts for device.encode_batch)."""
    out = []
    for c in cols:
        d = {"values": ctx.upload(c["values"]), "offset": c["offset"],
             "validity": ctx.upload(c["validity"]) if c["validity"] is not None else None,
             "offsets": ctx.upload(c["offsets"]) if c["offsets"] is not None else None,
             "utf8_bytes": int(c["offsets"][-1]) if c["offsets"] is not None else 0}
        out.append(d)
    return out


def oracle_cols(cols):
    """Buffer dicts in the oracle's encode_batch input format."""
    return [{"values": c["values"], "validity": c["validity"], "offsets": c["offsets"],
             "offset": c["offset"]} for c in cols]
