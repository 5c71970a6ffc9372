"""The oracle's MemoryStore restatement (oracle.MemStore: src/io/store/memory.rs
read / write over ReadBatchBuilder), the CPU baseline of a resident read
(bench.py --mode resident): a key's later write wins, a miss is an all-null
row, and the batch equals the builder fed the same rows in key order."""
import numpy as np

import oracle as O
from murr_amd import synth


def test_memstore_read_is_store_read():
    rng = np.random.default_rng(5)
    n = 3000
    cols = synth.config_c(n)
    dtypes = [int(c["dtype"]) for c in cols]
    seg = O.Segment(dtypes)
    blob, row_off = O.encode_batch(seg, synth.oracle_cols(cols), n)
    keys = [f"key{i}" for i in range(n)]
    keys[2000] = "key7"  # written again: row 2000 replaces row 7
    store = O.MemStore(keys, blob, row_off)
    q = [f"key{i}" for i in rng.integers(0, 3300, size=900)] + ["key7", "key2000", "", "nope"]
    proj = [11, 0, 12, 4, 9, 11]
    got = store.read(seg, proj, q)
    last = {k: i for i, k in enumerate(keys)}
    sel = [last.get(k) for k in q]
    parts, offs = [], [0]
    for r in sel:
        b = b"" if r is None else bytes(blob[int(row_off[r]):int(row_off[r + 1])])
        parts.append(b)
        offs.append(offs[-1] + len(b))
    want = O.decode_block(seg, proj, b"".join(parts), np.array(offs, np.uint64))
    assert sel[-4] == 2000 and sel[-3] is None  # "key7" -> its later row; "key2000" was overwritten
    for p in range(len(proj)):
        for f in ("length", "null_count", "values", "validity"):
            assert got[p][f] == want[p][f], (p, f)
        if got[p]["offsets"] is not None:
            assert np.array_equal(got[p]["offsets"], want[p]["offsets"]), p


def test_memstore_empty_read():
    seg = O.Segment([0, 10])
    store = O.MemStore([], b"", np.zeros(1, np.uint64))
    out = store.read(seg, [0, 1], [])
    assert [a["length"] for a in out] == [0, 0]
    out = store.read(seg, [1, 0], ["a", "b"])
    assert [a["null_count"] for a in out] == [2, 2]
