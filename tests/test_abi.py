"""The C-ABI library loads and exports exactly what include/murr_codec.h
declares; layout helpers agree with the oracle.  No compute calls (CPU only)."""
import ctypes as C
import subprocess

import pytest

import oracle as O
from murr_amd import _abi
from murr_amd.schema import DTypeName, SegmentSchema


def test_library_loads_and_exports_every_header_symbol():
    L = _abi.lib()
    syms = _abi.header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # the ctypes signature table covers the header one to one
    assert sorted(_abi.SIGNATURES) == syms


def test_plan_time_every_mirrors_header():
    import re
    m = re.search(r"#define MURR_PLAN_TIME_EVERY (\d+)", open(_abi.HEADER).read())
    assert m and int(m.group(1)) == _abi.PLAN_TIME_EVERY


def test_abi_version_mirrors_header_and_library():
    # murr_block_t grew to 40 bytes in round 5, so the version moved
    # to 2 and the loader refuses a library of another version
    import re
    m = re.search(r"#define MURR_ABI_VERSION (\d+)", open(_abi.HEADER).read())
    assert m and int(m.group(1)) == _abi.ABI_VERSION == 2
    assert _abi.lib().murr_abi_version() == _abi.ABI_VERSION
    assert C.sizeof(_abi.Block) == 40


def test_exports_are_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for s in _abi.header_symbols():
        assert s in exported, s  # unmangled extern "C"


def test_library_targets_gfx950_only():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readobj", "--sections", _abi.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_dtype_sizes_match_reference():
    # src/io/codec/<dtype>.rs `fn size`
    want = {"Utf8": 4, "Bool": 1, "Int8": 1, "Int16": 2, "Int32": 4, "Int64": 8, "UInt8": 1,
            "UInt16": 2, "UInt32": 4, "UInt64": 8, "Float32": 4, "Float64": 8}
    for name, sz in want.items():
        assert DTypeName[name].size() == sz
    assert _abi.lib().murr_dtype_size(99) == -1


@pytest.mark.parametrize("dtypes", [
    ["float32"], ["float32", "utf8"], ["utf8", "utf8"],
    ["bool", "int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64", "float32",
     "float64", "utf8", "utf8", "float32", "float64", "int64"],
    ["float32"] * 10, [], ["int8"] * 9,
])
def test_segment_layout_matches_oracle(dtypes):
    seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
    oseg = O.Segment(dtypes)
    assert seg.bitset_size == oseg.bitset_size == (len(dtypes) + 7) // 8
    assert seg.capacity == oseg.capacity
    for i, c in enumerate(seg.columns):
        assert (c.index, c.offset) == (oseg._cols[i].index, oseg._cols[i].offset)


def test_bitmap_bytes_padded_to_words():
    L = _abi.lib()
    assert [L.murr_bitmap_bytes(n) for n in (0, 1, 8, 64, 65, 100000)] == [0, 8, 8, 8, 16, 12504]


def test_status_strings():
    assert _abi.status_str(_abi.E_INVALID_UTF8) == "invalid utf8"
    assert _abi.status_str(0) == "ok"


def test_no_device_reports_cleanly_on_cpu_host():
    n = C.c_int(-1)
    _abi.lib().murr_device_count(C.byref(n))
    assert n.value >= 0
