"""Device key index + gather (murr_index.hip through the C ABI) and
ResidentTable.read, against the store semantics the reference tests pin:
caller order with misses as all-null rows (src/io/store/rocksdb/mod.rs:368-399,
src/io/store/memory.rs:71-165), request column order and duplicates
(src/io/table/mod.rs:248-462), later writes of a key winning (memory.rs:47-56).

The expected side is (i) a dict restatement of MemoryStore (key -> last row)
over the written Arrow arrays and (ii) the builder path (Table over
MemoryStore, itself parity-tested against the oracle), compared buffer by
buffer."""
import numpy as np
import pyarrow as pa
import pytest

from murr_amd.device import set_default_opts

from murr_amd import ColumnSchema, DTypeName as D, TableSchema
from murr_amd.resident import ROW_MISSING, DeviceIndex, ResidentTable
from murr_amd.row import default_context
from murr_amd.store import MemoryStore
from murr_amd.table import Table
from murr_amd import synth

pytestmark = pytest.mark.gpu

C_DTYPES = [D.Bool, D.Int8, D.Int16, D.Int32, D.Int64, D.UInt8, D.UInt16, D.UInt32, D.UInt64,
            D.Float32, D.Float64, D.Utf8, D.Utf8, D.Float32, D.Float64, D.Int64]


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel_mode(request):
    set_default_opts(kernel=request.param)
    yield request.param
    set_default_opts()


def schema_c():
    cols = {"key": ColumnSchema(D.Utf8, False)}
    for i, d in enumerate(C_DTYPES):
        cols[f"c{i}"] = ColumnSchema(d)
    return TableSchema("key", cols)


def batch_c(n, start=0, seed=42, keys=None):
    cols = synth.config_c(n, start=start, seed_nulls=seed)
    arrays = [pa.array(keys if keys is not None else [f"key{start + i}" for i in range(n)], pa.string())]
    arrays += [synth.to_arrow(c) for c in cols]
    return pa.RecordBatch.from_arrays(arrays, names=["key"] + [f"c{i}" for i in range(len(C_DTYPES))])


def expected(batches, keys, columns):
    """MemoryStore restatement: key -> last written row; misses all-null."""
    whole = pa.Table.from_batches(batches).combine_chunks()
    last = {}
    for i, k in enumerate(whole.column("key").to_pylist()):
        last[k] = i
    idx = [last.get(k) for k in keys]
    take = pa.array(idx, pa.int64())
    return pa.RecordBatch.from_arrays([whole.column(c).combine_chunks().take(take) for c in columns],
                                      names=columns)


def assert_same(got, want):
    assert got.schema.names == want.schema.names
    for a, b in zip(got.columns, want.columns):
        assert a.equals(b), (a, b)


def test_index_lookup_rows_and_misses():
    ctx = default_context()
    keys = pa.array([f"k{i}" for i in range(5000)], pa.string())
    ix = DeviceIndex(ctx, keys)
    n, slots = ix.info()
    assert n == 5000 and slots >= 10000 and slots & (slots - 1) == 0
    q = ["k0", "k4999", "nope", "k17", "", "k17", "k5000"]
    assert ix.lookup(q).tolist() == [0, 4999, ROW_MISSING, 17, ROW_MISSING, 17, ROW_MISSING]
    assert ix.lookup([]).tolist() == []


def test_index_later_duplicate_wins():
    ctx = default_context()
    ks = ["a", "b", "a", "c", "b", "a"]
    ix = DeviceIndex(ctx, pa.array(ks, pa.string()))
    assert ix.lookup(["a", "b", "c", "d"]).tolist() == [5, 4, 3, ROW_MISSING]


def test_index_edge_keys():
    ctx = default_context()
    rng = np.random.default_rng(5)
    ks = ["", "x", "x" * 300, "xy", "yx", "éè", "pre" * 50 + "1", "pre" * 50 + "2"]
    ks += ["".join(chr(97 + c) for c in rng.integers(0, 3, size=int(rng.integers(1, 6)))) for _ in range(200)]
    uniq = list(dict.fromkeys(ks))
    last = {k: i for i, k in enumerate(ks)}
    ix = DeviceIndex(ctx, pa.array(ks, pa.string()))
    assert ix.lookup(uniq + ["zzz"]).tolist() == [last[k] for k in uniq] + [ROW_MISSING]


def test_index_all_rows_permutation_1m():
    # size-independent property at scale: every key finds its own row
    ctx = default_context()
    n = 1_000_000
    keys = pa.array([str(i) for i in range(n)], pa.string())
    ix = DeviceIndex(ctx, keys)
    rng = np.random.default_rng(9)
    perm = rng.permutation(n)
    rows = ix.lookup([str(i) for i in perm])
    assert np.array_equal(rows, perm.astype(np.uint32))


def test_resident_read_matches_store_semantics():
    t = ResidentTable(schema_c())
    b0 = batch_c(20000, seed=42)
    t.write(b0)
    rng = np.random.default_rng(44)
    ids = rng.integers(0, 21000, size=3000)  # ~5% misses
    keys = [f"key{i}" for i in ids]
    cols = [f"c{i}" for i in range(16)]
    got = t.read(keys, cols)
    assert_same(got, expected([b0], keys, cols))
    # request order, duplicates, subset
    cols2 = ["c11", "c0", "c11", "c15", "c12"]
    assert_same(t.read(keys[:777], cols2), expected([b0], keys[:777], cols2))


def test_resident_read_bit_exact_vs_builder_path():
    ts = schema_c()
    b0 = batch_c(5000, seed=7)
    rt = ResidentTable(ts)
    rt.write(b0)
    mt = Table.create(MemoryStore(), "t", ts)
    mt.write(b0)
    rng = np.random.default_rng(8)
    keys = [f"key{i}" for i in rng.integers(0, 5300, size=1000)]
    cols = [f"c{i}" for i in range(16)]
    got, want = rt.read(keys, cols), mt.read(keys, cols)
    for a, b in zip(got.columns, want.columns):
        ba, bb = a.buffers(), b.buffers()
        assert a.null_count == b.null_count
        for x, y in zip(ba[1:], bb[1:]):
            assert x.to_pybytes() == y.to_pybytes()
        if a.null_count:
            nb = (len(a) + 7) // 8
            assert ba[0].to_pybytes()[:nb] == bb[0].to_pybytes()[:nb]


def test_resident_overwrite_and_append():
    t = ResidentTable(schema_c())
    b0 = batch_c(3000, seed=1)
    b1 = batch_c(1500, start=2000, seed=2)  # keys 2000..3499: 1000 overwrite, 500 new
    t.write(b0)
    t.write(b1)
    keys = [f"key{i}" for i in (0, 1999, 2000, 2999, 3000, 3499, 3500)]
    cols = [f"c{i}" for i in range(16)]
    assert_same(t.read(keys, cols), expected([b0, b1], keys, cols))


def test_resident_all_miss_and_empty_query():
    t = ResidentTable(schema_c())
    t.write(batch_c(100))
    got = t.read(["x", "y", "z"], ["c3", "c11"])
    assert got.num_rows == 3 and all(c.null_count == 3 for c in got.columns)
    got = t.read([], ["c3", "c11"])
    assert got.num_rows == 0


def test_resident_table_schema_errors():
    from murr_amd.errors import SegmentError
    t = ResidentTable(schema_c())
    t.write(batch_c(10))
    with pytest.raises(SegmentError):
        t.read(["key1"], ["key"])
    with pytest.raises(SegmentError):
        t.read(["key1"], ["nope"])


def test_resident_read_many_keys_three_pass_scan():
    # > 4096 queries: probe, three scan passes over 4096-query groups, copy
    t = ResidentTable(schema_c())
    b0 = batch_c(30000, seed=3)
    t.write(b0)
    rng = np.random.default_rng(11)
    keys = [f"key{i}" for i in rng.integers(0, 31500, size=20000)]
    cols = ["c12", "c4", "c0", "c11"]
    assert_same(t.read(keys, cols), expected([b0], keys, cols))


@pytest.mark.parametrize("nk,cap,with_rows", [(1500, 5000, True), (700, 5000, True), (1024, 20000, False),
                                               (1024, 300000, True), (1, 16, False), (64, 100000, False)])
def test_gather_capacity_clamp(nk, cap, with_rows):
    # out_cap too small: offsets clamp to the cap, `needed` reports the size.
    # nk <= 1024 takes the spread probe + per-workgroup scan copy
    # (gather_probe_wide / gather_scan_copy), above it the one-workgroup scan.
    # Every fifth key misses; rows NULL puts them in the context's scratch.
    from murr_amd.resident import _upload_utf8
    t = ResidentTable(schema_c())
    t.write(batch_c(2000, seed=4))
    ctx = t.ctx
    want_rows = [i if i % 5 else 10**9 for i in range(nk)]
    keys = [f"key{r}" for r in want_rows]
    qd, qo = _upload_utf8(ctx, pa.array(keys, pa.string()))
    data, offs, needed = ctx.alloc(cap + 16), ctx.alloc((nk + 1) * 8), ctx.alloc(8)
    rows = ctx.alloc(nk * 4) if with_rows else None
    st = ctx.L.murr_index_gather(ctx.h, t.index.h, qd.ptr, qo.ptr, nk, t.blob.ptr, t.row_off.ptr,
                                 data.ptr, cap, offs.ptr, rows.ptr if rows else None, needed.ptr)
    assert st == 0
    off = offs.download((nk + 1) * 8).view(np.uint64)
    full = t.row_off.download((t.n + 1) * 8).view(np.uint64)
    sizes = np.array([int(full[r + 1] - full[r]) if r < t.n else 0 for r in want_rows], np.uint64)
    want = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    assert int(needed.download(8).view(np.uint64)[0]) == int(want[-1])
    assert np.array_equal(off, np.minimum(want, cap))
    if rows:
        assert rows.download(nk * 4).view(np.uint32).tolist() == \
            [r if r < t.n else ROW_MISSING for r in want_rows]
    blob = t.blob.download(int(full[-1]))
    exp = b"".join(blob[int(full[r]):int(full[r + 1])].tobytes() for r in want_rows if r < t.n)
    got = data.download(cap)
    k = int(np.searchsorted(want, cap, side="right")) - 1  # rows wholly inside the cap
    assert got[:int(want[k])].tobytes() == exp[:int(want[k])]


def test_index_long_duplicate_keys():
    # multi-chunk keys (> 32 B) through the insert's equal-key path
    ctx = default_context()
    base = "k" * 95
    ks = [base + "a", base + "b", base + "a", "z" * 64, base + "b", "z" * 64, "z" * 65]
    ix = DeviceIndex(ctx, pa.array(ks, pa.string()))
    assert ix.lookup([base + "a", base + "b", "z" * 64, "z" * 65, base + "c", "z" * 63]).tolist() == \
        [2, 4, 5, 6, ROW_MISSING, ROW_MISSING]


def test_incremental_appends_keep_earlier_rows_and_later_write_wins():
    # MemoryStore::write appends (src/io/store/memory.rs:47-60): each write
    # encodes only its batch onto the arena tail (earlier rows' blobs and
    # offsets stay byte-identical) and a key written again maps to its new row
    ctx = default_context()
    rt = ResidentTable(schema_c(), ctx)
    batches = []
    rng = np.random.default_rng(17)
    prev_off = None
    for w in range(6):
        n = int(rng.integers(1, 3000))
        # half new keys, half rewrites of keys from earlier batches
        keys = [f"key{w * 100000 + i}" for i in range(n)]
        if w:
            for i in rng.choice(n, size=n // 2, replace=False):
                keys[i] = f"key{int(rng.integers(0, w)) * 100000 + int(rng.integers(0, 50))}"
        b = batch_c(n, start=w * 1000, seed=w, keys=keys)
        n_before, used_before = rt.n, rt.used
        rt.write(b)
        batches.append(b)
        assert rt.n == n_before + n
        off = rt.row_off.download(8 * (rt.n + 1)).view(np.uint64)
        assert int(off[n_before]) == used_before and int(off[-1]) == rt.used
        if prev_off is not None:
            assert np.array_equal(off[:len(prev_off)], prev_off)  # earlier rows untouched
        prev_off = off.copy()
        q = [f"key{int(x)}" for x in rng.integers(0, (w + 1) * 100000, size=300)]
        q += [k for k in rng.choice(keys, size=200)]
        cols = [f"c{i}" for i in rng.permutation(len(C_DTYPES))[:9]]
        assert_same(rt.read(q, cols), expected(batches, q, cols))


def test_oversized_row_sizes_the_gather_exactly():
    # one 64 KiB string: keys x longest row is far above the single-phase
    # bound, so the gather looks the rows up first and allocates exactly
    ctx = default_context()
    rt = ResidentTable(schema_c(), ctx)
    n = 3000
    b = batch_c(n, seed=3)
    arrays = list(b.columns)
    big = arrays[12].to_pylist()
    big[7] = "x" * 65536
    arrays[12] = pa.array(big, pa.string())
    b = pa.RecordBatch.from_arrays(arrays, names=b.schema.names)
    rt.write(b)
    assert rt.max_row > 65536
    rng = np.random.default_rng(9)
    q = [f"key{int(x)}" for x in rng.integers(0, n + 100, size=5000)] + ["key7"] * 3
    from murr_amd import resident
    assert len(q) * rt.max_row > resident.TWO_PHASE_BYTES
    cols = [f"c{i}" for i in range(len(C_DTYPES))]
    assert_same(rt.read(q, cols), expected([b], q, cols))


def test_reference_bench_dataset_chunked_reads():
    """The read benches' table (benches/common/dataset.rs:24-55, col_j = i as f32,
    key = i.to_string()) written in chunks like bench.py --mode resident --table ref,
    read with keys sampled as benches/common/read_bench.rs:89-98 (1000 keys per
    read, uniform over the rows): every key hits and every column is `i as f32`."""
    n, chunk = 250_000, 60_000
    t = ResidentTable(synth.ref_schema())
    batches = []
    for s in range(0, n, chunk):
        batches.append(synth.ref_batch(s, min(chunk, n - s)))
        t.write(batches[-1])
    cols = [f"col_{j}" for j in range(10)]
    for k in range(3):
        ids = np.random.default_rng(1000 * 2_000_000 + k).integers(0, n, size=1000)
        keys = [str(int(i)) for i in ids]
        got = t.read(keys, cols)
        want = ids.astype(np.float32)
        for c in got.columns:
            assert c.null_count == 0
            assert np.array_equal(c.to_numpy(), want)
        assert_same(got, expected(batches, keys, cols))
    # projection subset and the largest key
    got = t.read([str(n - 1), "0", str(n)], ["col_9", "col_0"])
    assert got.column(0).to_pylist() == [float(n - 1), 0.0, None]
