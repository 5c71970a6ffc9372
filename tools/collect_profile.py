"""Copy a round profile (tools/round_profile.sh output under gpurun_out/$R)
into profiles/$R: bench lines as JSON, rocprofv3 kernel stats, and the
FETCH_SIZE / WRITE_SIZE passes summarised per dispatch (KiB)."""
import csv
import glob
import json
import os
import shutil
import sys

R = sys.argv[1] if len(sys.argv) > 1 else "r02"
src = f"gpurun_out/{R}"
dst = f"profiles/{sys.argv[2]}" if len(sys.argv) > 2 else f"profiles/{R}"  # (e.g. r05f -> r05)
os.makedirs(dst, exist_ok=True)


def last_json(path):
    line = None
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = ln
    return json.loads(line) if line else None


names = {"bench": "bench.json", "decode_C": "decode_C.json", "decode_D1": "decode_D1.json",
         "host_B": "host_B.json", "encode_E": "encode_E.json", "decode_C_noindex": "decode_C_noindex.json",
         "decode_D10M": "decode_D10M.json", "decode_D1_noindex": "decode_D1_noindex.json",
         "decode_B_generic": "decode_B_generic.json", "host_C": "host_C.json", "encode_B": "encode_B.json",
         "encode_C": "encode_C.json", "resident_1000": "resident_1000.json",
         "resident_read_plain": "resident_read_plain.json", "resident_read_block": "resident_read_block.json",
         "decode_D1x2": "decode_D1x2.json", "decode_D1x4": "decode_D1x4.json",
         "decode_D_table10M": "decode_D_table10M.json", "sst": "sst_bench.json"}
for n, out in names.items():
    p = f"{src}/{n}.log"
    if os.path.exists(p):
        j = last_json(p)
        if j is not None:
            json.dump(j, open(f"{dst}/{out}", "w"))
            print(out)
if os.path.exists(f"{src}/trace.log"):  # the traced driver command's own line
    j = last_json(f"{src}/trace.log")
    if j is not None:
        open(f"{dst}/bench_driver_traced_line.log", "w").write(json.dumps(j) + "\n")
        print("bench_driver_traced_line.log")
for n in ("timeline_D",):
    if os.path.exists(f"{src}/{n}.log"):
        shutil.copy(f"{src}/{n}.log", f"{dst}/{n}.log")
        print(f"{n}.log")
for pat, out in [("trace/*kernel_stats.csv", "bench_driver_kernel_stats.csv"),
                 ("trace/*domain_stats.csv", "bench_driver_domain_stats.csv"),
                 ("trace_res_C/*kernel_stats.csv", "resident_C_100reads_kernel_stats.csv")]:
    f = sorted(glob.glob(f"{src}/{pat}"))
    if f:
        shutil.copy(f[0], f"{dst}/{out}")
        print(out)
f = sorted(glob.glob(f"{src}/trace/*kernel_trace.csv"))
if f:  # the headline's launches apart from the lanes run's overlapped ones
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "trace_split.py"),
                          f[0]], capture_output=True, text=True).stdout
    open(f"{dst}/bench_driver_kernel_split.txt", "w").write(out)
    print("bench_driver_kernel_split.txt")
for c in ("B", "C"):
    f = sorted(glob.glob(f"gpurun_out/encprof/{c}/*kernel_stats.csv"))
    if f:
        shutil.copy(f[0], f"{dst}/encode_{c}_kernel_stats.csv")
        print(f"encode_{c}_kernel_stats.csv")
rows = []
for f in sorted(glob.glob(f"{src}/pmc/*counter_collection.csv")):
    run = os.path.basename(f).replace("_counter_collection.csv", "")
    per = {}
    for r in csv.DictReader(open(f)):
        if "decode" not in r["Kernel_Name"]:
            continue
        k = (r["Counter_Name"], r["Kernel_Name"], r["Dispatch_Id"])
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    for (cn, kn, d), v in sorted(per.items(), key=lambda x: int(x[0][2])):
        rows.append([run, cn, kn, d, f"{v:.6f}"])
if rows:
    with open(f"{dst}/pmc_traffic.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["run", "counter", "kernel", "dispatch", "value_kib"])
        w.writerows(rows)
    print("pmc_traffic.csv")
