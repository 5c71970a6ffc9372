"""The prepared resident read (murr_read_plan_*, ResidentTable.read's path):
lookup + gather + decode (+ the arrays to pinned memory) enqueued once and
waited for once.  Checked against the MemoryStore restatement of
src/io/store/memory.rs:28-45 (a miss is an all-null row), against the
builder path bit for bit, and against round 5's unprepared device path, at key
counts around the plan's capacity classes (a run of nq keys decodes
read_capacity(nq) rows, the rest misses)."""
import ctypes as C

import numpy as np
import pyarrow as pa
import pytest

from murr_amd import _abi
from murr_amd.device import DecodeOutputs, DeviceBlock, decode_blocks, download_array
from murr_amd.resident import ReadPlan, ResidentTable, _upload_utf8, read_capacity
from murr_amd.store import MemoryStore
from murr_amd.table import Table

from test_gpu_resident import assert_same, batch_c, expected, schema_c

pytestmark = pytest.mark.gpu

COLS = [f"c{i}" for i in range(16)]


@pytest.fixture(scope="module")
def table():
    rt = ResidentTable(schema_c())
    b0 = batch_c(6000, seed=42)
    rt.write(b0)
    return rt, b0


def test_capacity_classes():
    assert [read_capacity(n) for n in (1, 63, 64, 65, 1000, 1024, 1025, 5000)] == \
        [64, 64, 64, 128, 1024, 1024, 2048, 8192]


@pytest.mark.parametrize("nq", [1, 5, 63, 64, 65, 700, 1000, 1025, 3000])
def test_plan_reads_match_store_semantics(table, nq):
    rt, b0 = table
    rng = np.random.default_rng(1000 + nq)
    keys = [f"key{i}" for i in rng.integers(0, 6300, size=nq)]  # ~5 % misses
    got = rt.read(keys, COLS)
    assert_same(got, expected([b0], keys, COLS))
    plan = rt.read_plan(COLS, nq)
    assert isinstance(plan, ReadPlan) and plan.cap == read_capacity(nq)
    assert rt.ctx.L.murr_read_plan_capacity(plan.h) == plan.cap


def test_plan_bit_exact_vs_builder_path(table):
    rt, b0 = table
    mt = Table.create(MemoryStore(), "t", schema_c())
    mt.write(b0)
    rng = np.random.default_rng(8)
    keys = [f"key{i}" for i in rng.integers(0, 6300, size=1000)]
    got, want = rt.read(keys, COLS), mt.read(keys, COLS)
    for a, b in zip(got.columns, want.columns):
        ba, bb = a.buffers(), b.buffers()
        assert a.null_count == b.null_count
        for x, y in zip(ba[1:], bb[1:]):
            assert x.to_pybytes() == y.to_pybytes()
        if a.null_count:
            nb = (len(a) + 7) // 8
            assert ba[0].to_pybytes()[:nb] == bb[0].to_pybytes()[:nb]


def test_plan_reused_across_key_sets_and_replaced_after_a_write():
    rt = ResidentTable(schema_c())
    b0 = batch_c(3000, seed=3)
    rt.write(b0)
    rng = np.random.default_rng(9)
    cols = ["c11", "c0", "c15", "c12"]
    k1 = [f"key{i}" for i in rng.integers(0, 3200, size=900)]
    k2 = [f"key{i}" for i in rng.integers(0, 3200, size=1000)]
    assert_same(rt.read(k1, cols), expected([b0], k1, cols))
    p1 = rt.read_plan(cols, 900)
    assert_same(rt.read(k2, cols), expected([b0], k2, cols))
    assert rt.read_plan(cols, 1000) is p1  # same class (1024), same table state: reused
    # a write (overwrites and new keys) changes the table: a new plan, the new rows
    b1 = batch_c(1500, start=2500, seed=4)
    rt.write(b1)
    k3 = [f"key{i}" for i in rng.integers(0, 4100, size=1000)]
    assert_same(rt.read(k3, cols), expected([b0, b1], k3, cols))
    assert rt.read_plan(cols, 1000) is not p1 and p1.h is None  # (the stale plan was freed)
    # a plan held across a write is closed by the write itself: running it
    # raises instead of reading the arena the write may have moved
    p2 = rt.read_plan(cols, 1000)
    rt.write(batch_c(10, start=9000, seed=5))
    assert p2.h is None
    from murr_amd import SegmentError
    with pytest.raises(SegmentError):
        p2.run(pa.array(k3[:1000], pa.string()))


def test_plan_keys_as_sliced_arrow_array_and_all_misses(table):
    rt, b0 = table
    allk = pa.array([f"key{i}" for i in range(0, 6600, 3)], pa.string())
    q = allk.slice(100, 500)
    assert_same(rt.read(q, COLS), expected([b0], q.to_pylist(), COLS))
    miss = ["nope", "", "key-1", "key99999"]
    assert_same(rt.read(miss, ["c3", "c11"]), expected([b0], miss, ["c3", "c11"]))
    assert rt.read([], ["c3", "c11"]).num_rows == 0


def test_plan_device_run_equals_unprepared_path(table):
    # the device variant (keys in HBM, arrays in HBM) against round 5's two-call
    # path (murr_index_gather + murr_decode_blocks) on the same keys
    rt, _ = table
    ctx, L = rt.ctx, rt.ctx.L
    rng = np.random.default_rng(77)
    nq = 1000
    keys = pa.array([f"key{i}" for i in rng.integers(0, 6300, size=nq)], pa.string())
    qd, qo = _upload_utf8(ctx, keys)
    plan = rt.read_plan(COLS, nq)
    dev = plan.run_device(qd.ptr, qo.ptr, nq)
    blk, _keep = rt.gather(keys.to_pylist())
    proj = [c.index for c in rt._resolve(COLS)]
    outs = DecodeOutputs(ctx, rt.segment, proj, [blk])
    decode_blocks(ctx, rt.segment, proj, [blk], outs)
    for p, ci in enumerate(proj):
        dt = int(rt.segment.columns[ci].dtype)
        a, b = download_array(ctx, dev[p], dt, nq), download_array(ctx, outs.array(0, p), dt, nq)
        assert a["null_count"] == b["null_count"], p
        assert a["values"] == b["values"], p
        if dt == 0:
            assert np.array_equal(a["offsets"], b["offsets"]), p
        if a["null_count"]:
            nb = (nq + 7) // 8
            assert a["validity"][:nb] == b["validity"][:nb], p


def test_row_lengths_match_the_written_strings(table):
    # murr_utf8_row_lengths, kept by ResidentTable beside its arena: per row
    # and utf8 column, the string bytes the decode's offsets advance by (0 for
    # a null cell)
    rt, b0 = table
    assert rt.nutf8 == 2 and rt.ulen is not None
    got = rt.ulen.download(4 * 2 * rt.n).view(np.uint32).reshape(rt.n, 2)
    for u, name in enumerate(["c11", "c12"]):
        want = [len(s.encode()) if s is not None else 0 for s in b0.column(name).to_pylist()]
        assert got[:, u].tolist() == want, name


@pytest.mark.parametrize("nq,mode", [(1, "cut"), (700, "cut"), (1000, "cut"), (1024, "cut"), (3000, "split")])
def test_plan_indexes_its_gather_up_to_1024_keys(table, nq, mode):
    # up to 1024 keys the gather writes the gathered block's utf8 index and
    # the decode cuts the block (one pass); above, split mode (two passes)
    rt, b0 = table
    rng = np.random.default_rng(31 + nq)
    keys = [f"key{i}" for i in rng.integers(0, 6300, size=nq)]
    assert_same(rt.read(keys, COLS), expected([b0], keys, COLS))
    assert rt.ctx.stats()["last_mode"] == mode


def test_plan_five_utf8_columns_takes_split_mode():
    # more utf8 columns than the gather indexes (4): the decode splits the block
    from murr_amd import ColumnSchema, DTypeName as D, TableSchema
    cols = {"key": ColumnSchema(D.Utf8, False)}
    for i in range(5):
        cols[f"s{i}"] = ColumnSchema(D.Utf8)
    cols["v"] = ColumnSchema(D.Int32)
    rt = ResidentTable(TableSchema("key", cols))
    rng = np.random.default_rng(5)
    n = 3000
    arrays = [pa.array([f"key{i}" for i in range(n)], pa.string())]
    for i in range(5):
        arrays.append(pa.array([None if rng.random() < 0.2 else "x" * int(rng.integers(0, 40)) for _ in range(n)],
                               pa.string()))
    arrays.append(pa.array(rng.integers(-5, 5, size=n).astype(np.int32)))
    b = pa.RecordBatch.from_arrays(arrays, names=["key"] + [f"s{i}" for i in range(5)] + ["v"])
    rt.write(b)
    assert rt.ulen is None
    names = [f"s{i}" for i in range(5)] + ["v"]
    keys = [f"key{i}" for i in rng.integers(0, 3100, size=1000)]
    assert_same(rt.read(keys, names), expected([b], keys, names))
    assert rt.ctx.stats()["last_mode"] == "split"


@pytest.mark.parametrize("nu", [1, 3, 4])
def test_plan_index_from_row_lengths_any_utf8_count(nu):
    # layouts of 1, 3 and 4 utf8 columns (with empty, null and long strings,
    # some over 1 KiB) between fixed-width ones: the gather's utf8 index from
    # the per-row string bytes, a one-pass decode, the MemoryStore's answer;
    # then an append (the row lengths extend) and a read over both batches
    from murr_amd import ColumnSchema, DTypeName as D, TableSchema
    rng = np.random.default_rng(70 + nu)
    cols = {"key": ColumnSchema(D.Utf8, False), "a": ColumnSchema(D.Int64)}
    for i in range(nu):
        cols[f"s{i}"] = ColumnSchema(D.Utf8)
    cols["b"] = ColumnSchema(D.Bool)
    rt = ResidentTable(TableSchema("key", cols))
    names = ["a"] + [f"s{i}" for i in range(nu)] + ["b"]

    def batch(start, n):
        arrays = [pa.array([f"key{start + i}" for i in range(n)], pa.string()),
                  pa.array(rng.integers(-10**12, 10**12, size=n).astype(np.int64))]
        for _ in range(nu):
            vals = []
            for _ in range(n):
                r = rng.random()
                vals.append(None if r < 0.15 else "" if r < 0.25 else
                            "y" * int(rng.integers(1000, 3000)) if r < 0.27 else
                            "é" * int(rng.integers(1, 20)))
            arrays.append(pa.array(vals, pa.string()))
        arrays.append(pa.array([None if rng.random() < 0.1 else bool(rng.random() < 0.5) for _ in range(n)]))
        return pa.RecordBatch.from_arrays(arrays, names=["key"] + names)

    b0 = batch(0, 4000)
    rt.write(b0)
    assert rt.ulen is not None
    for nq in (1, 333, 1000):
        keys = [f"key{i}" for i in rng.integers(0, 4200, size=nq)]
        assert_same(rt.read(keys, names), expected([b0], keys, names))
        assert rt.ctx.stats()["last_mode"] == "cut"
    b1 = batch(3500, 2000)  # overwrites 500 keys, adds 1500
    rt.write(b1)
    keys = [f"key{i}" for i in rng.integers(0, 5600, size=1000)]
    assert_same(rt.read(keys, names), expected([b0, b1], keys, names))
    assert rt.ctx.stats()["last_mode"] == "cut"


def test_plan_soak_reads_between_appends():
    # many prepared reads of random sizes (every capacity class up to 2048,
    # so both gather forms and both decode modes) between appends that
    # overwrite and add keys, each checked against the MemoryStore
    # restatement: the fused gather's alternating look-back word sets, the
    # plans' reuse and their invalidation by a write, over many cycles
    rt = ResidentTable(schema_c())
    rng = np.random.default_rng(2026)
    batches = []
    start = 0
    for cycle in range(5):
        m = int(rng.integers(500, 2500))
        keys = [f"key{start + i}" for i in range(m)]
        for i in rng.choice(m, size=m // 4, replace=False):  # overwrites of earlier keys
            if start:
                keys[i] = f"key{int(rng.integers(0, start))}"
        b = batch_c(m, start=start, seed=cycle, keys=keys)
        rt.write(b)
        batches.append(b)
        start += m
        cols = [f"c{i}" for i in rng.permutation(16)[:int(rng.integers(1, 17))]]
        for _ in range(40):
            nq = int(rng.choice([1, 2, 63, 64, 65, 200, 511, 700, 1000, 1024, 1025, 2048]))
            q = [f"key{int(x)}" for x in rng.integers(0, int(start * 1.05) + 1, size=nq)]
            assert_same(rt.read(q, cols), expected(batches, q, cols))


def test_plan_slot_cache_long_and_short_keys():
    # the index's slot cache (murr_index_cache_rows, kept by every write):
    # keys of <= 16 bytes resolve on the slot's key prefix, longer ones
    # compare their remaining bytes; overwrites move a key's slot to its new
    # row, a rehash rebuilds the cache; all against the MemoryStore restatement
    rt = ResidentTable(schema_c())
    rng = np.random.default_rng(616)

    def key(i):
        return f"key{i}" if i % 3 else f"a-longer-key-of-the-table-{i:08d}"  # 4-10 or 34 bytes

    batches, start = [], 0
    for w, m in enumerate([700, 1500, 5000]):  # the second and third appends rehash
        keys = [key(start + i) for i in range(m)]
        if start:
            for i in rng.choice(m, size=m // 5, replace=False):
                keys[i] = key(int(rng.integers(0, start)))
        b = batch_c(m, start=start, seed=w, keys=keys)
        rt.write(b)
        batches.append(b)
        start += m
        for nq in (1, 100, 1000):
            q = [key(int(x)) for x in rng.integers(0, int(start * 1.05), size=nq)] + ["a-longer-key-of-the-table-x"]
            assert_same(rt.read(q, COLS), expected(batches, q, COLS))


def test_plan_keys_at_their_length_bounds():
    # keys of every length 1 .. 40 around the probe's bounds (the slot
    # cache's 16-byte key prefix, the 32-byte key chunk; 28 bytes: the 32-B
    # key record of EXPERIMENTS #30), multi-byte text, a 28-byte miss and the
    # empty key, each read against the MemoryStore restatement
    rt = ResidentTable(schema_c())
    rng = np.random.default_rng(28)

    def key(i):
        n = i % 41
        return ("é" * (n // 2) + "k" * (n % 2)) if i % 7 == 0 else (f"{i:x}" * 41)[:n]

    keys = sorted({key(i) for i in range(4000)} - {""}, key=lambda s: (len(s.encode()), s))
    keys = [k for k in keys if len(k.encode()) <= 40]
    b = batch_c(len(keys), seed=6, keys=keys)
    rt.write(b)
    short = [k for k in keys if len(k.encode()) <= 28]
    assert any(len(k.encode()) == 28 for k in short) and any(len(k.encode()) == 17 for k in short)
    for nq in (1, 64, 1000):
        q = [short[int(x)] for x in rng.integers(0, len(short), size=nq)]
        q[-1] = "k" * 28 if nq > 1 else q[-1]  # (a 28-byte miss)
        assert_same(rt.read(q, COLS), expected([b], q, COLS))
        q2 = q[:-1] + [keys[-1]]  # (one key of 40 bytes: two key chunks)
        assert len(keys[-1].encode()) > 28
        assert_same(rt.read(q2, COLS), expected([b], q2, COLS))
    assert_same(rt.read([""], COLS), expected([b], [""], COLS))
