#!/usr/bin/env bash
# Per-row instruction / wait counters of the decode kernel for a few
# projections (one rocprofv3 --pmc pass per counter group; no trace domains).
set -u
export TMPDIR=/tmp
out=gpurun_out/pmcr
mkdir -p $out
for pj in ${PJS:-1 0}; do
 i=0
 while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $counters --output-format csv -d $out -o p${pj/,/_}_$i -- python3 bench.py --steps 2 --warmup 1 --no-cpu --proj $pj > $out/p${pj/,/_}_$i.log 2>&1 || { echo "pass $pj/$i failed"; tail -5 $out/p${pj/,/_}_$i.log; exit 1; }
 done <<LIST
${PMC_LIST:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT}
LIST
done
python3 - <<'PY'
import csv, glob, collections, re
rows = 100_000_000
for tag in sorted({re.sub(r"_\d+_counter.*", "", f.split("/")[-1]) for f in glob.glob("gpurun_out/pmcr/*_counter_collection.csv")}):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pmcr/{tag}_*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "decode" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(tag)
    for k, v in sorted(agg.items()):
        m = sum(v.values()) / len(v)
        print(f"  {k:28s} {m:14.4g}   per64rows {m / (rows / 64):10.2f}")
PY
