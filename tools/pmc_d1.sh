#!/usr/bin/env bash
# PMC passes over the config-D one-shard decode (split mode), for the
# instruction mix and wait breakdown of the decode kernel.
set -u
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcD1}
ARGS=${BENCH_ARGS:-"--config D --steps 3 --warmup 1 --no-cpu"}
mkdir -p $OUT
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
                "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
                "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d $OUT -o pass$i -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass$i exit=$rc"
  [ $rc -eq 0 ] || exit $rc
done
