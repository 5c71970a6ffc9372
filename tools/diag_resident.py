import sys; sys.path.insert(0, "tests")
import numpy as np
from test_gpu_resident import *
ts = schema_c(); b0 = batch_c(5000, seed=7)
rt = ResidentTable(ts); rt.write(b0)
mt = Table.create(MemoryStore(), "t", ts); mt.write(b0)
rng = np.random.default_rng(8)
keys = [f"key{i}" for i in rng.integers(0, 5300, size=1000)]
cols = [f"c{i}" for i in range(16)]
got, want = rt.read(keys, cols), mt.read(keys, cols)
for ci, (a, b) in enumerate(zip(got.columns, want.columns)):
    print(ci, a.type, "eq", a.equals(b), a.null_count, b.null_count)
    for bi, (x, y) in enumerate(zip(a.buffers()[1:], b.buffers()[1:])):
        xb, yb = x.to_pybytes(), y.to_pybytes()
        if xb != yb:
            d = next((i for i in range(min(len(xb), len(yb))) if xb[i] != yb[i]), None)
            print("  buf", bi + 1, "len", len(xb), len(yb), "first diff", d, xb[d:d+8] if d is not None else b"", yb[d:d+8] if d is not None else b"")
