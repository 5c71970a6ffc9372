import numpy as np, pyarrow as pa
from murr_amd.resident import DeviceIndex, ROW_MISSING
from murr_amd.row import default_context
ctx = default_context()
rng = np.random.default_rng(5)
ks = ["", "x", "x" * 300, "xy", "yx", "éè", "pre" * 50 + "1", "pre" * 50 + "2"]
ks += ["".join(chr(97 + c) for c in rng.integers(0, 3, size=int(rng.integers(1, 6)))) for _ in range(200)]
uniq = list(dict.fromkeys(ks))
last = {k: i for i, k in enumerate(ks)}
want = [last[k] for k in uniq] + [ROW_MISSING]
for rep in range(3):
    ix = DeviceIndex(ctx, pa.array(ks, pa.string()))
    for r2 in range(2):
        got = ix.lookup(uniq + ["zzz"]).tolist()
        bad = [(i, uniq[i][:12] if i < len(uniq) else "zzz", g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
        print(rep, r2, "bad", bad[:8])
    for single in ["x" * 300, "pre" * 50 + "1", "x"]:
        print("  single", len(single), ix.lookup([single]).tolist(), last[single])
