#!/usr/bin/env bash
# SQ / TA / TD passes over the config-C encode kernel.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_enc
mkdir -p $OUT
i=0
for counters in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
                "SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
                "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT -o pass$i -- python3 bench.py --mode encode --enc-config C --steps 3 --warmup 1 > $OUT/pass$i.log 2>&1
  echo "pass$i exit=$?"
done
python3 tools/pmc_sum.py $OUT murr_jit_encode
