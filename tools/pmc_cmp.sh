set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
for dbg in 3 4; do
 i=0
 for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"; do
  i=$((i+1))
  MURR_DEBUG_DECODE=$dbg timeout -k 10 200 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc2 -o d${dbg}_p$i -- python3 bench.py --steps 2 --warmup 1 --no-cpu --proj 1 > gpurun_out/pmc2/d${dbg}_p$i.log 2>&1 || exit $?
 done
done
python3 - <<'PY'
import csv, glob, collections
for dbg in (3, 4):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(f"gpurun_out/pmc2/d{dbg}_p*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "decode_kernel" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print("dbg", dbg, " ".join(f"{k}={sum(v.values())/len(v):.3g}" for k, v in sorted(agg.items())))
PY
