"""configs[0] (benches/read_plain.rs on CPU: 1k rows, one FLOAT32 column)
through the CPU restatement: oracle encode -> oracle decode is the closed form
f = i, and the blob layout is the reference's (bitset byte 0xFE: bit 0 clear = not null, then
the f32 little-endian; src/io/row/write.rs:19-52)."""
import numpy as np

import oracle as O
from murr_amd import synth
from murr_amd.schema import DTypeName as D


def test_config_a_oracle_roundtrip():
    n = 1000
    cols = synth.config_a(n)
    seg = O.Segment([int(D.Float32)])
    blob, off = O.encode_batch(seg, synth.oracle_cols(cols), n)
    assert np.array_equal(np.diff(off.astype(np.int64)), np.full(n, 5))
    rows = blob.reshape(n, 5)
    assert (rows[:, 0] == 0xFE).all()  # bitset starts all-null (0xFF); bit 0 cleared for the value
    assert np.array_equal(rows[:, 1:].copy().view(np.float32).ravel(), np.arange(n, dtype=np.float32))
    out = O.decode_block(seg, [0], blob, off)[0]
    assert out["null_count"] == 0
    assert np.array_equal(np.frombuffer(out["values"], np.float32), np.arange(n, dtype=np.float32))
