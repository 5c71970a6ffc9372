"""Instruction mix of one kernel in a hipcc -S listing (tuning aid)."""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
body, on = [], False
for line in open(path):
    if line.startswith(name + ":"):
        on = True
        continue
    if on:
        if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
            break
        s = line.strip()
        if s and not s.startswith((".", ";")) and not s.endswith(":"):
            body.append(s.split()[0])
c = Counter()
for m in body:
    k = ("s_" if m.startswith("s_") else "ds_" if m.startswith("ds_") else "global/buffer" if m.startswith(("global_", "buffer_", "flat_")) else "v_")
    c[k] += 1
print(len(body), dict(c))
top = Counter(body).most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25)
print(top)
