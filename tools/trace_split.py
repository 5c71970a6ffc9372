"""Split a bench trace's decode dispatches (rocprofv3 --kernel-trace CSV) into
the headline's single-stream launches and the `lanes` run's overlapped ones,
so the rocprof average of the headline kernel can be set beside the bench
line's kernel_ms_avg (bench.py times the headline's launches alone; its lanes
key runs 3 streams whose launches overlap and each take longer).
usage: trace_split.py <kernel_trace.csv> [warmup] [steps]"""
import csv
import sys

path = sys.argv[1]
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith("murr_jit_decode")]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
solo, over = [], []
for i, (s, e, k) in enumerate(iv):
    o = any(not (e2 <= s or s2 >= e) for j, (s2, e2, _) in enumerate(iv) if j != i)
    (over if o else solo).append((e - s) / 1e6)
timed = solo[warm:warm + steps]
avg = lambda v: sum(v) / len(v) if v else 0.0
print(f"{iv[0][2] if iv else '-'}: {len(iv)} dispatches")
print(f"  single-stream launches: {len(solo)}, avg {avg(solo):.4f} ms")
print(f"  the headline's timed launches (single-stream {warm}..{warm + steps - 1}): avg {avg(timed):.4f} ms, "
      f"min {min(timed) if timed else 0:.4f}, max {max(timed) if timed else 0:.4f}")
print(f"  overlapped launches (the lanes run, 3 streams): {len(over)}, avg {avg(over):.4f} ms each")
