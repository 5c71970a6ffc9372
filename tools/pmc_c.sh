#!/usr/bin/env bash
# Instruction / wait counters of the decode kernel on one config (default C).
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcc}
ARGS=${BENCH_ARGS:-"--config C --blocks 10 --steps 2 --warmup 1 --no-cpu"}
mkdir -p $OUT
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $counters --output-format csv -d $OUT -o p$i -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT
FETCH_SIZE
WRITE_SIZE
LIST
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{out}/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "decode" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"  {k:28s} {sum(v.values()) / len(v):14.5g}")
PY
