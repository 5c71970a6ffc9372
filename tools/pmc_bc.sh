#!/usr/bin/env bash
# SQ instruction-mix / wait passes for decode B and C, then encode kernel stats.
set -u
export TMPDIR=/tmp
for cfg in "B:--steps 3 --warmup 1 --no-cpu" "C:--config C --blocks 10 --steps 3 --warmup 1 --no-cpu"; do
  n=${cfg%%:*}; a=${cfg#*:}
  OUT=gpurun_out/pmc_$n
  mkdir -p $OUT
  i=0
  for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
                  "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d $OUT -o pass$i -- python3 bench.py $a > $OUT/pass$i.log 2>&1
    rc=$?
    echo "$n pass$i exit=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_sum.py $OUT murr_jit_decode
done
bash tools/enc_prof.sh
