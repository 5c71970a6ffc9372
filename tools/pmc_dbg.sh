#!/usr/bin/env bash
# VALU/SALU/LDS instruction counts per 64 rows for decode ablations (DBGS list).
set -u
export TMPDIR=/tmp
out=gpurun_out/pmcd
mkdir -p $out
for d in ${DBGS:-0 4}; do
  MURR_DEBUG_DECODE=$d MURR_DECODE_TILE_BYTES=${TB:-16384} timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $out -o d$d -- python3 bench.py --steps 2 --warmup 1 --no-cpu --proj ${PJ:-0} > $out/d$d.log 2>&1 || { echo "dbg $d failed"; tail -5 $out/d$d.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
rows = 100_000_000
for d in os.environ.get("DBGS", "0 4").split():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pmcd/d{d}_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "decode_kernel" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print("dbg", d, " ".join(f"{k[9:]}={sum(v.values())/len(v)/(rows/64):.1f}" for k, v in sorted(agg.items())))
PY
