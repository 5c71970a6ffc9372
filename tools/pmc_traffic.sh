#!/usr/bin/env bash
# HBM traffic and memory-pipe counters of the headline decode (one rocprofv3
# --pmc pass per group, no trace domains), summarised per launch.
set -u
export TMPDIR=/tmp
out=gpurun_out/pmct
mkdir -p $out
rocprofv3 -L > $out/counters.txt 2>&1 || true
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $out -o t_$i -- python3 bench.py --steps 2 --warmup 1 --no-cpu ${ARGS:-} > $out/t_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/t_$i.log; exit 1; }
done <<LIST
${PMC_LIST:-FETCH_SIZE
WRITE_SIZE
TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE
TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_COUNT}
LIST
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmct/t_*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "decode" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"  {k:32s} {sum(v.values()) / len(v):14.6g}")
PY
