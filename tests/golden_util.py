"""Helpers shared by the parity tests: golden fixture loading and Arrow-buffer
comparison (bit-exact, including null slots and bitmap padding)."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DTYPE_CODES = {"utf8": 0, "bool": 1, "int8": 2, "int16": 3, "int32": 4, "int64": 5,
               "uint8": 6, "uint16": 7, "uint32": 8, "uint64": 9, "float32": 10, "float64": 11}
SIZES = {0: 4, 1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 1, 7: 2, 8: 4, 9: 8, 10: 4, 11: 8}


def load_cases(*files):
    files = files or ("rows.json", "dtypes.json", "tables.json", "parquet.json")
    out = []
    for f in files:
        with open(os.path.join(GOLDEN, f)) as fh:
            out += json.load(fh)["cases"]
    return out


def block_from_rows(rows):
    """rows: list of hex strings or None (missing key) -> (data u8, row_off u64)."""
    parts, off = [], [0]
    for r in rows:
        b = bytes.fromhex(r) if r is not None else b""
        parts.append(b)
        off.append(off[-1] + len(b))
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy(), np.array(off, dtype=np.uint64)


def expected_array(e):
    return {"dtype": DTYPE_CODES[e["dtype"]], "length": e["length"], "null_count": e["null_count"],
            "values": bytes.fromhex(e["values"]),
            "validity": bytes.fromhex(e["validity"]) if e["validity"] else None,
            "offsets": np.array(e["offsets"], dtype=np.int32) if e["offsets"] is not None else None}


def encode_inputs(case):
    cols = []
    for e in case["encode_input"]:
        a = expected_array(e)
        cols.append({"values": a["values"], "validity": a["validity"], "offsets": a["offsets"],
                     "offset": 0})
    return cols


def assert_array_equal(got, exp, ctx=""):
    """Bit-exact Arrow comparison of buffer dicts."""
    n = exp["length"]
    assert got["length"] == n, f"{ctx}: length {got['length']} != {n}"
    assert got["null_count"] == exp["null_count"], f"{ctx}: null_count {got['null_count']} != {exp['null_count']}"
    if exp["validity"] is None:
        assert got["validity"] is None, f"{ctx}: unexpected validity buffer"
    else:
        nb = (n + 7) // 8
        assert got["validity"] is not None, f"{ctx}: validity missing"
        assert bytes(got["validity"][:nb]) == exp["validity"], f"{ctx}: validity differs"
    dt = exp["dtype"]
    if dt == 0:
        go = np.asarray(got["offsets"], dtype=np.int32)
        assert np.array_equal(go[: n + 1], exp["offsets"]), f"{ctx}: offsets differ"
        assert bytes(got["values"][: int(exp["offsets"][-1])]) == exp["values"], f"{ctx}: utf8 data differs"
    elif dt == 1:
        nb = (n + 7) // 8
        assert bytes(got["values"][:nb]) == exp["values"], f"{ctx}: bool bits differ"
    else:
        w = SIZES[dt]
        assert bytes(got["values"][: n * w]) == exp["values"], f"{ctx}: values differ"
