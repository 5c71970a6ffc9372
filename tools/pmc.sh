#!/usr/bin/env bash
# PMC counter passes over a short decode bench (one rocprofv3 per pass; no trace
# domains combined with --pmc).  Outputs under gpurun_out/pmc/.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu"}
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d $OUT -o pass$i -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass$i ($counters) exit=$rc"
  case $rc in 0) ;; *) exit $rc ;; esac
done <<LIST
${PMC_LIST:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM
SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT
FETCH_SIZE
WRITE_SIZE
TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT}
LIST
