"""Seeded random workloads for the parity tests (test infrastructure)."""
from __future__ import annotations

import numpy as np

from murr_amd import synth
from murr_amd.schema import DTypeName as D

ALL = list(D)
NP = {D.Int8: np.int8, D.Int16: np.int16, D.Int32: np.int32, D.Int64: np.int64, D.UInt8: np.uint8,
      D.UInt16: np.uint16, D.UInt32: np.uint32, D.UInt64: np.uint64, D.Float32: np.float32,
      D.Float64: np.float64}


def random_columns(rng, dtypes, n, null_p=0.1, max_str=24, unicode=True, long_every=0,
                   long_len=40000):
    cols = []
    for dt in dtypes:
        valid = rng.random(n) >= null_p if null_p else np.ones(n, bool)
        if dt == D.Utf8:
            lens = rng.integers(0, max_str + 1, size=n)
            if long_every:
                lens[::long_every] = long_len
            lens = lens * valid
            parts = []
            for L in lens:
                if unicode and L >= 3 and rng.random() < 0.3:
                    s = ("é" * (L // 2)).encode()[:L]
                    s = s[: len(s) - (len(s) % 2)]
                    s = s + b"x" * (L - len(s))
                else:
                    s = rng.integers(0x20, 0x7F, size=L, dtype=np.uint8).tobytes()
                parts.append(s)
            offs = np.zeros(n + 1, np.int64)
            np.cumsum([len(p) for p in parts], out=offs[1:])
            data = np.frombuffer(b"".join(parts), np.uint8).copy()
            cols.append(synth.column(dt, valid=valid, offsets=offs.astype(np.int32), data=data, n=n))
        elif dt == D.Bool:
            cols.append(synth.column(dt, rng.random(n) < 0.5, valid))
        else:
            raw = rng.integers(0, 256, size=n * np.dtype(NP[dt]).itemsize, dtype=np.uint8)
            v = raw.view(NP[dt]).copy()  # any bit pattern, NaNs included for floats
            v[~valid] = 0
            cols.append(synth.column(dt, v, valid))
    return cols


def drop_rows(data, row_off, missing):
    """Turn rows whose index is in `missing` into empty rows (missing keys)."""
    parts, off = [], [0]
    for i in range(len(row_off) - 1):
        b = b"" if i in missing else data[int(row_off[i]):int(row_off[i + 1])].tobytes()
        parts.append(b)
        off.append(off[-1] + len(b))
    return np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(off, np.uint64)
