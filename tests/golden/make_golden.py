"""Generate the golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

The reference (murrdb/murr v0.2.1, Rust) cannot be built or imported here, so
the fixtures restate the reference's OWN known-answer tests as data:

* the row-format unit tests, src/io/row/write.rs:71-146, with blob bytes
  derived by hand from WriteRow (write.rs:19-52) and asserted below;
* every per-dtype rstest case of `assert_row_roundtrip`
  (src/io/codec/test_util.rs:23-46: Arrow -> ColumnDecoder -> WriteRow ->
  ReadRow -> ColumnEncoder -> Arrow must equal the input), e.g.
  src/io/codec/int8.rs:58-66, uint64.rs:58-67, float32.rs:58-66 and the NaN
  test float32.rs:82-105, bool_.rs:126-132, utf8.rs:141-148 and the invalid
  UTF-8 test utf8.rs:160-170;
* the store order/miss tests (src/io/store/rocksdb/mod.rs:368-424,
  src/io/store/memory.rs:101-146) and the table tests (src/io/table/mod.rs:230-462);
* util/example.parquet (a real data file shipped with the reference) as an
  encode/decode round-trip input.

This script is a second, independent restatement (Python) of the codec; the C
oracle (oracle/murr_oracle.c) is checked against these fixtures by
tests/test_oracle_golden.py.  Expected Arrow buffers follow arrow-rs 58 builder
semantics (null slots zero-filled, validity absent when there are no nulls,
LSB-first bitmaps with zero trailing bits, utf8 null = repeated offset) and are
cross-checked against pyarrow's logical values here.

Run:  python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
from __future__ import annotations

import json
import math
import os
import struct
import sys

import numpy as np
import pyarrow as pa

HERE = os.path.dirname(os.path.abspath(__file__))

# DTypeName order, src/core/schema.rs:6-19
DTYPES = ["utf8", "bool", "int8", "int16", "int32", "int64",
          "uint8", "uint16", "uint32", "uint64", "float32", "float64"]
SIZE = {"utf8": 4, "bool": 1, "int8": 1, "int16": 2, "int32": 4, "int64": 8,
        "uint8": 1, "uint16": 2, "uint32": 4, "uint64": 8, "float32": 4, "float64": 8}
FMT = {"int8": "<b", "int16": "<h", "int32": "<i", "int64": "<q",
       "uint8": "<B", "uint16": "<H", "uint32": "<I", "uint64": "<Q",
       "float32": "<f", "float64": "<d"}
PA_TYPE = {"utf8": pa.string(), "bool": pa.bool_(), "int8": pa.int8(), "int16": pa.int16(),
           "int32": pa.int32(), "int64": pa.int64(), "uint8": pa.uint8(), "uint16": pa.uint16(),
           "uint32": pa.uint32(), "uint64": pa.uint64(), "float32": pa.float32(),
           "float64": pa.float64()}


def segment(dtypes):
    """From<&TableSchema> for SegmentSchema (src/io/schema.rs:33-54)."""
    cols, off = [], 0
    for i, d in enumerate(dtypes):
        cols.append({"index": i, "dtype": d, "offset": off, "size": SIZE[d]})
        off += SIZE[d]
    return {"cols": cols, "bitset_size": (len(dtypes) + 7) // 8, "capacity": off}


def encode_value(dtype, v):
    """Native little-endian bytes (bytemuck::bytes_of); floats may be given as
    ('bits', int) to carry exact bit patterns such as NaN payloads."""
    if isinstance(v, tuple) and v[0] == "bits":
        return v[1].to_bytes(SIZE[dtype], "little")
    if dtype == "bool":
        return bytes([1 if v else 0])
    return struct.pack(FMT[dtype], v)


def write_row(seg, values):
    """WriteRow::new + ColumnDecoder::write_to_row per column (write.rs:20-52,
    primitive.rs:90-94, bool_.rs:112-116, utf8.rs:114-118).  None = Arrow null."""
    bs, cap = seg["bitset_size"], seg["capacity"]
    b = bytearray(bs + cap)
    b[:bs] = b"\xff" * bs
    for c, v in zip(seg["cols"], values):
        if v is None:
            continue
        b[c["index"] // 8] &= ~(1 << (c["index"] % 8)) & 0xFF
        at = bs + c["offset"]
        if c["dtype"] == "utf8":
            raw = v if isinstance(v, (bytes, bytearray)) else v.encode()
            rel = len(b) - bs
            b[at:at + 4] = struct.pack("<I", rel)
            b += struct.pack("<I", len(raw)) + raw
        else:
            b[at:at + c["size"]] = encode_value(c["dtype"], v)
    return bytes(b)


def bitmap(bits):
    out = bytearray((len(bits) + 7) // 8)
    for i, v in enumerate(bits):
        if v:
            out[i // 8] |= 1 << (i % 8)
    return bytes(out)


def arrow_buffers(dtype, values):
    """arrow-rs builder output for `values` (None = null)."""
    n = len(values)
    valid = [v is not None for v in values]
    nulls = n - sum(valid)
    out = {"dtype": dtype, "length": n, "null_count": nulls,
           "validity": bitmap(valid).hex() if nulls else None, "offsets": None}
    if dtype == "utf8":
        data, offs = bytearray(), [0]
        for v in values:
            if v is not None:
                data += v if isinstance(v, (bytes, bytearray)) else v.encode()
            offs.append(len(data))
        out["values"] = bytes(data).hex()
        out["offsets"] = offs
    elif dtype == "bool":
        out["values"] = bitmap([bool(v) for v in [x if x is not None else False for x in values]]).hex()
    else:
        out["values"] = b"".join(encode_value(dtype, v) if v is not None else b"\0" * SIZE[dtype]
                                 for v in values).hex()
    return out


def pa_check(expected, values):
    """Cross-check the restated buffers against pyarrow's logical values."""
    dt = expected["dtype"]
    bufs = [pa.py_buffer(bytes.fromhex(expected["validity"])) if expected["validity"] else None]
    if dt == "utf8":
        bufs += [pa.py_buffer(np.array(expected["offsets"], dtype=np.int32).tobytes()),
                 pa.py_buffer(bytes.fromhex(expected["values"]))]
    else:
        bufs += [pa.py_buffer(bytes.fromhex(expected["values"]))]
    arr = pa.Array.from_buffers(PA_TYPE[dt], expected["length"], bufs,
                                null_count=expected["null_count"])
    arr.validate(full=True)
    got = arr.to_pylist()
    for g, v in zip(got, values):
        if v is None:
            assert g is None
        elif isinstance(v, tuple):
            pass  # bit patterns (NaN) checked bitwise by the tests
        elif dt == "utf8":
            assert g == (v.decode() if isinstance(v, bytes) else v), (g, v)
        elif dt.startswith("float") and isinstance(v, float) and math.isnan(v):
            assert math.isnan(g)
        else:
            assert g == v, (g, v)


def case(name, source, dtypes, rows_values, proj=None, expect_error=None, missing=()):
    """rows_values: per row a list of per-column values (None = null); rows whose
    index is in `missing` are absent keys (empty blob -> add_empty)."""
    seg = segment(dtypes)
    proj = list(range(len(dtypes))) if proj is None else proj
    blobs = [None if i in missing else write_row(seg, r) for i, r in enumerate(rows_values)]
    c = {"name": name, "source": source, "dtypes": dtypes, "proj": proj,
         "rows": [b.hex() if b is not None else None for b in blobs],
         "expect_error": expect_error}
    # Arrow input for the encode direction (all rows present).
    c["encode_input"] = [arrow_buffers(d, [r[j] for r in rows_values]) for j, d in enumerate(dtypes)]
    if expect_error is None:
        exp = []
        for p in proj:
            vals = [None if i in missing else r[p] for i, r in enumerate(rows_values)]
            e = arrow_buffers(dtypes[p], vals)
            pa_check(e, vals)
            exp.append(e)
        c["expected"] = exp
    # Encode output (all rows present); omitted when identical to "rows".
    all_blobs = [write_row(seg, r) for r in rows_values]
    c["encode_blobs"] = [b.hex() for b in all_blobs] if missing else None
    return c


def known_answer_rows():
    """src/io/row/write.rs:71-146, with blob bytes derived by hand."""
    cases = []
    # roundtrip_static_f32_f64 (write.rs:71-85): bitset 0xFF & ~0b11 = 0xFC,
    # 1.5f32 = 0x3FC00000, -3.25f64 = 0xC00A000000000000.
    c = case("row_static_f32_f64", "src/io/row/write.rs:71-85",
             ["float32", "float64"], [[1.5, -3.25]])
    assert c["rows"][0] == "fc" + "0000c03f" + "0000000000000ac0", c["rows"][0]
    cases.append(c)
    # roundtrip_dynamic_utf8 (write.rs:87-101): slot a = 9-1 = 8, payload len 0;
    # slot b = 13-1 = 12, payload len 10 "δ-unicode".
    c = case("row_dynamic_utf8", "src/io/row/write.rs:87-101",
             ["utf8", "utf8"], [[b"", "δ-unicode".encode()]])
    assert c["rows"][0] == ("fc" + "08000000" + "0c000000" + "00000000" + "0a000000"
                            + "δ-unicode".encode().hex()), c["rows"][0]
    cases.append(c)
    # roundtrip_mixed_f32_utf8 (write.rs:103-119): 42.5f32 = 0x422A0000; slot = 8.
    c = case("row_mixed_f32_utf8", "src/io/row/write.rs:103-119",
             ["float32", "utf8"], [[42.5, b"hello"]])
    assert c["rows"][0] == "fc" + "00002a42" + "08000000" + "05000000" + b"hello".hex()
    cases.append(c)
    # roundtrip_with_nulls (write.rs:121-146): both / only_float / none.
    c = case("row_with_nulls", "src/io/row/write.rs:121-146",
             ["float32", "utf8"], [[1.0, b"hi"], [7.5, None], [None, None]])
    assert c["rows"][1] == "fe" + "0000f040" + "00000000"  # only bit 0 cleared
    assert c["rows"][2] == "ff" + "00000000" + "00000000"
    cases.append(c)
    return cases


def dtype_roundtrips():
    """Every assert_row_roundtrip rstest case, one single-row block each, plus
    all cases of a dtype stacked into one block."""
    table = {
        # src/io/codec/int8.rs:58-66 etc.: neg/null/min/max/zero
        "int8": [-7, None, -128, 127, 0],
        "int16": [-7, None, -(1 << 15), (1 << 15) - 1, 0],
        "int32": [-7, None, -(1 << 31), (1 << 31) - 1, 0],
        "int64": [-7, None, -(1 << 63), (1 << 63) - 1, 0],
        # uint*.rs:58-66: null/zero/max/mid; uint64.rs:63 adds 2^53+1
        "uint8": [None, 0, 255, 7],
        "uint16": [None, 0, 65535, 7],
        "uint32": [None, 0, (1 << 32) - 1, 7],
        "uint64": [None, 0, (1 << 64) - 1, 7, (1 << 53) + 1],
        # float32.rs:58-66 pos/null/neg/zero; float64.rs same
        "float32": [1.5, None, -2.5, 0.0],
        "float64": [1.5, None, -2.5, 0.0],
        # bool_.rs:126-132 t/null/f
        "bool": [True, None, False],
        # utf8.rs:141-148 ascii/null/empty/unicode
        "utf8": [b"hello", None, b"", "δ-unicode".encode()],
    }
    src = {"int8": "src/io/codec/int8.rs:58-66", "int16": "src/io/codec/int16.rs:58-66",
           "int32": "src/io/codec/int32.rs:58-66", "int64": "src/io/codec/int64.rs:58-66",
           "uint8": "src/io/codec/uint8.rs:58-66", "uint16": "src/io/codec/uint16.rs:58-66",
           "uint32": "src/io/codec/uint32.rs:58-66", "uint64": "src/io/codec/uint64.rs:58-67",
           "float32": "src/io/codec/float32.rs:58-66", "float64": "src/io/codec/float64.rs:58-66",
           "bool": "src/io/codec/bool_.rs:126-132", "utf8": "src/io/codec/utf8.rs:141-148"}
    cases = []
    for dt, vals in table.items():
        for k, v in enumerate(vals):
            cases.append(case(f"roundtrip_{dt}_{k}", src[dt], [dt], [[v]]))
        cases.append(case(f"roundtrip_{dt}_all", src[dt], [dt], [[v] for v in vals]))
    # float32.rs:82-105: NaN must survive bit-exactly (quiet NaN + a payload NaN).
    cases.append(case("roundtrip_float32_nan", "src/io/codec/float32.rs:82-105", ["float32"],
                      [[("bits", 0x7FC00000)], [("bits", 0xFFA00001)], [("bits", 0x7F800001)]]))
    cases.append(case("roundtrip_float64_nan", "src/io/codec/float32.rs:82-105 (f64 analogue)",
                      ["float64"], [[("bits", 0x7FF8000000000000)], [("bits", 0xFFF0000000000001)]]))
    # utf8.rs:160-170: invalid UTF-8 payload -> SegmentError.
    cases.append(case("utf8_invalid", "src/io/codec/utf8.rs:160-170", ["utf8"],
                      [[bytes([0xFF, 0xFE, 0xFD])]], expect_error="invalid_utf8"))
    # More invalid forms under core::str::from_utf8 (overlong, surrogate, > U+10FFFF, truncated).
    for k, bad in enumerate([b"\xc0\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"ab\xe2\x82",
                             b"\x80", b"ok\xf0\x9f\x98"]):
        cases.append(case(f"utf8_invalid_{k}", "core::str::from_utf8 (utf8.rs:90-92 call site)",
                          ["utf8"], [[b"fine"], [bad]], expect_error="invalid_utf8"))
    # Valid multi-byte forms at the range edges.
    cases.append(case("utf8_valid_edges", "core::str::from_utf8 (utf8.rs:90-92 call site)", ["utf8"],
                      [[b"\xc2\x80"], [b"\xdf\xbf"], [b"\xe0\xa0\x80"], [b"\xed\x9f\xbf"],
                       [b"\xee\x80\x80"], [b"\xf0\x90\x80\x80"], [b"\xf4\x8f\xbf\xbf"],
                       ["😀".encode()]]))
    return cases


def store_and_table_cases():
    cases = []
    # store order with a miss: rocksdb/mod.rs:368-399 (payload_segment = one utf8 col,
    # src/io/store/test_util.rs:9-16).  Looked-up order dave, alice, zzz, carol, bob.
    cases.append(case("store_caller_order_with_miss", "src/io/store/rocksdb/mod.rs:368-399",
                      ["utf8"], [[b"d"], [b"a"], [None], [b"c"], [b"b"]], missing=(2,)))
    cases.append(case("store_missing_key", "src/io/store/memory.rs:124-146",
                      ["utf8"], [[b"a-payload"], [None], [b"c-payload"]], missing=(1,)))
    # table/mod.rs:230-246 roundtrip_writes_and_reads_back (score: f32 with a null)
    cases.append(case("table_roundtrip_score", "src/io/table/mod.rs:230-246",
                      ["float32"], [[1.0], [None], [3.0]]))
    # table/mod.rs:248-302 projection order: segment (score f32, label utf8)
    cases.append(case("table_request_order_label_score", "src/io/table/mod.rs:248-302",
                      ["float32", "utf8"], [[1.0, b"x"], [2.0, b"y"]], proj=[1, 0]))
    cases.append(case("table_request_order_score_label", "src/io/table/mod.rs:248-302",
                      ["float32", "utf8"], [[1.0, b"x"], [2.0, b"y"]], proj=[0, 1]))
    # table/mod.rs:338-349 missing key -> null
    cases.append(case("table_missing_key", "src/io/table/mod.rs:338-349",
                      ["float32"], [[1.0], [None]], missing=(1,)))
    # table/mod.rs:380-462 mixed f32/f64/utf8 with nulls
    cases.append(case("table_mixed_dtypes", "src/io/table/mod.rs:380-462",
                      ["float32", "float64", "utf8"],
                      [[1.5, None, b"x"], [None, 2.0, None], [-2.5, 3.0, b"z"]]))
    # duplicate projection (ReadBatchBuilder keeps request order incl. duplicates, read.rs:74-77)
    cases.append(case("duplicate_projection", "src/io/row/read.rs:69-83",
                      ["float32", "utf8"], [[1.0, b"x"], [None, b"yy"]], proj=[1, 1, 0]))
    # C > 8: multi-byte bitset (16 columns, config C dtype order)
    c16 = ["bool", "int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64",
           "float32", "float64", "utf8", "utf8", "float32", "float64", "int64"]
    rows = []
    for r in range(70):  # > 64 rows: crosses a wave / bitmap word
        row = []
        for j, d in enumerate(c16):
            if (r * 7 + j * 3) % 10 == 0:
                row.append(None)
            elif d == "utf8":
                row.append(("%d" % (r * 31 + j)).encode() * ((r + j) % 4))
            elif d == "bool":
                row.append((r + j) % 3 == 0)
            elif d.startswith("float"):
                row.append(r * 0.5 - j)
            elif d.startswith("u"):
                row.append((r * 977 + j) % (1 << (8 * SIZE[d])))
            else:
                lim = 1 << (8 * SIZE[d] - 1)
                row.append(((r * 977 + j) % (2 * lim)) - lim)
        rows.append(row)
    cases.append(case("config_c_schema_70_rows", "BASELINE.json configs[2] schema; src/io/schema.rs:33-54",
                      c16, rows, proj=[15, 0, 11, 3, 12, 9, 9, 1], missing=(5, 64, 69)))
    return cases


def parquet_case():
    """util/example.parquet: key utf8 (RocksDB key) + value int64 (util/generate_parquet.py:4-8)."""
    import pyarrow.parquet as pq
    t = pq.read_table(os.path.join(HERE, "example.parquet"))
    vals = t.column("value").to_pylist()
    return case("example_parquet_int64", "util/example.parquet (reference data file)",
                ["int64"], [[v] for v in vals])


def main():
    groups = {
        "rows.json": known_answer_rows(),
        "dtypes.json": dtype_roundtrips(),
        "tables.json": store_and_table_cases(),
        "parquet.json": [parquet_case()],
    }
    for fname, cases in groups.items():
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f, indent=None,
                      separators=(",", ":"))
        print(f"{fname}: {len(cases)} cases", file=sys.stderr)


if __name__ == "__main__":
    main()
