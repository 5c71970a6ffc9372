"""Per-dispatch averages of PMC counters for kernels matching a pattern
(a substring, or the whole name when the pattern ends with '$')."""
import csv
import glob
import sys
from collections import defaultdict

d, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "murr_jit_decode"
vals = defaultdict(list)
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if (name == pat[:-1]) if pat.endswith("$") else (pat in name):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, cn), v in per.items():
        vals[cn].append(v)
for cn, v in sorted(vals.items()):
    print(f"{cn:24s} {sum(v) / len(v):16.0f}  (n={len(v)})")
