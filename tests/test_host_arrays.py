"""Host Arrow assembly of a read (murr_amd.row.host_arrays_to_arrow: copies of
the output region's runs, zero-copy slices, descriptors read as one numpy
view; host_arrays_to_batch: the library's Arrow C Data Interface export,
murr_arrow_export, imported in one call) equals the per-column conversion,
buffer for buffer (CPU: synthetic murr_host_array_t over a host region laid
out as the library's)."""
import numpy as np
import pytest

from murr_amd import _abi
from murr_amd.row import c_names, host_array_to_arrow, host_arrays_to_arrow, host_arrays_to_batch
from murr_amd.schema import DTypeName as D


@pytest.mark.parametrize("n", [0, 1, 7, 64, 1000])
@pytest.mark.parametrize("gap", [64, 1 << 16])  # packed region, or one whose span is mostly gaps
def test_batched_equals_per_column(n, gap):
    rng = np.random.default_rng(n + gap)
    region = np.zeros(16 * (n * 8 + gap + 256), np.uint8)
    base = region.ctypes.data
    off = [0]

    def put(arr):
        b = np.frombuffer(arr.tobytes(), np.uint8)
        o = off[0]
        region[o:o + len(b)] = b
        off[0] = (o + len(b) + gap + 63) // 64 * 64
        return base + o

    dtypes = [D.Utf8, D.Float32, D.Int64, D.Bool, D.UInt8, D.Utf8, D.Int16, D.Float64]
    outs = (_abi.HostArray * len(dtypes))()
    for i, dt in enumerate(dtypes):
        h = outs[i]
        if dt == D.Utf8:
            lens = rng.integers(0, 9, n)
            o = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
            d = rng.integers(97, 123, int(o[-1]), dtype=np.uint8)
            h.offsets, h.values, h.values_len = put(o), put(d) if len(d) else base, len(d)
        else:
            nb = (n + 7) // 8 if dt == D.Bool else n * {D.Float32: 4, D.Int64: 8, D.UInt8: 1, D.Int16: 2, D.Float64: 8}[dt]
            v = rng.integers(0, 256, nb, dtype=np.uint8)
            if dt == D.Bool and n % 8:
                v[-1] &= 0xFF >> (8 - n % 8)
            h.offsets, h.values, h.values_len = None, put(v) if nb else base, nb
        h.dtype = int(dt)
        if i % 2 == 0 and n:
            bits = rng.integers(0, 256, (n + 7) // 8, dtype=np.uint8)
            if n % 8:
                bits[-1] &= 0xFF >> (8 - n % 8)
            h.validity = put(bits)
            h.null_count = int(n - np.unpackbits(bits, bitorder="little")[:n].sum())
        else:
            h.validity, h.null_count = None, 0
        h.length = n
    want = [host_array_to_arrow(outs[i]) for i in range(len(dtypes))]
    # the Arrow C Data Interface export (murr_arrow_export) imported as one
    # RecordBatch: the same arrays, named, nullable, buffer for buffer
    names = [f"col{i}" for i in range(len(dtypes))]
    rb = host_arrays_to_batch(outs, len(dtypes), c_names(names))
    rb.validate(full=True)
    assert rb.schema.names == names and all(f.nullable for f in rb.schema)
    for i, (x, y) in enumerate(zip(rb.columns, want)):
        assert x.type == y.type and len(x) == len(y) and x.null_count == y.null_count, i
        for bx, by in zip(x.buffers(), y.buffers()):
            assert (bx is None) == (by is None), i
            if bx is not None:
                assert bx.to_pybytes() == by.to_pybytes(), i
    # against the schema of an earlier export (no schema side exported): the same batch
    rb2 = host_arrays_to_batch(outs, len(dtypes), c_names(names), rb.schema)
    rb2.validate(full=True)
    assert rb2.schema == rb.schema and rb2.num_rows == rb.num_rows  # (random floats: NaNs, so bytes below)
    for x, y in zip(rb2.columns, rb.columns):
        for bx, by in zip(x.buffers(), y.buffers()):
            assert (bx is None) == (by is None) and (bx is None or bx.to_pybytes() == by.to_pybytes())
    del rb, rb2  # (released through the export's callbacks)
    got = host_arrays_to_arrow(outs, len(dtypes))
    for i, (x, y) in enumerate(zip(got, [host_array_to_arrow(outs[i]) for i in range(len(dtypes))])):
        x.validate(full=True)
        assert x.type == y.type and len(x) == len(y) and x.null_count == y.null_count, i  # (random floats: NaNs)
        for bx, by in zip(x.buffers(), y.buffers()):
            assert (bx is None) == (by is None)
            if bx is not None:
                assert bx.to_pybytes() == by.to_pybytes()


def test_arrow_export_rejects_mixed_lengths_and_releases():
    import ctypes as C
    import gc
    a = np.arange(10, dtype=np.int32)
    outs = (_abi.HostArray * 2)()
    for h, n in zip(outs, (10, 9)):
        h.values, h.values_len, h.length, h.dtype = a.ctypes.data, 4 * n, n, int(D.Int32)
    arr, sch = _abi.ArrowArray(), _abi.ArrowSchema()
    assert _abi.lib().murr_arrow_export(outs, 2, c_names(["a", "b"]), C.byref(arr), C.byref(sch)) == _abi.E_ARGUMENT
    outs[1].length, outs[1].values_len = 10, 40
    rbs = [host_arrays_to_batch(outs, 2, c_names(["a", "b"])) for _ in range(200)]
    assert all(r.column(1).to_pylist() == list(range(10)) for r in rbs)
    del rbs
    gc.collect()
