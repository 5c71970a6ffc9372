#!/usr/bin/env python3
"""Per-launch durations and the gaps between consecutive launches of one
kernel from a rocprofv3 --kernel-trace CSV (…_kernel_trace.csv).

  python tools/trace_gaps.py TRACE.csv [KERNEL_SUBSTRING]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "decode"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if want in r.get("Kernel_Name", ""):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    prev = None
    durs, gaps = [], []
    for s, e, n in rows:
        d = (e - s) / 1e3
        g = (s - prev) / 1e3 if prev is not None else float("nan")
        durs.append(d)
        if prev is not None:
            gaps.append(g)
        print(f"{n:40s} start {s} dur {d:9.2f} us  gap {g:8.2f} us")
        prev = e
    if durs:
        print(f"launches {len(durs)}  mean dur {sum(durs) / len(durs):.2f} us  "
              f"mean gap {sum(gaps) / max(len(gaps), 1):.2f} us")


if __name__ == "__main__":
    main()
