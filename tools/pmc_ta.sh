#!/usr/bin/env bash
# Memory-pipeline counters (TA / TD / TCP) for decode B; lists the gfx950
# counter names first.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ta
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1 || true
grep -oE "\b(TA|TD|TCP|TCC)_[A-Z0-9_]+" $OUT/list.txt | sort -u > $OUT/names.txt || true
wc -l $OUT/names.txt
i=0
for counters in "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d $OUT -o pass$i -- python3 bench.py ${ARGS:---steps 3 --warmup 1 --no-cpu} > $OUT/pass$i.log 2>&1
  echo "pass$i ($counters) exit=$?"
done
python3 tools/pmc_sum.py $OUT murr_jit_decode
