#!/usr/bin/env bash
# Counter passes over one bench.py configuration: one rocprofv3 --pmc pass per
# counter group (never combined with a trace domain, each pass bounded), then
# per-dispatch averages of the kernels matching $KERNEL (tools/pmc_sum.py).
#   OUT=gpurun_out/pmcX KERNEL=murr_jit_decode ARGS="--config C --blocks 10" bash tools/pmc_passes.sh
# Groups: SQ occupancy / issue, SQ instruction mix, memory pipeline, HBM bytes.
# The interpreter goes after `--` by its resolved path: rocprofv3 execs it,
# and a `python3` found on PATH may be a wrapper that execs again.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
OUT=${OUT:-gpurun_out/pmc}
KERNEL=${KERNEL:-murr_jit_decode}
ARGS=${ARGS:---steps 3 --warmup 1}
mkdir -p "$OUT"
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES" \
            "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
            ${EXTRA_GROUPS:-} "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT" -o pass$i -- \
    "$PY" bench.py $ARGS --no-cpu --no-traffic > "$OUT/pass$i.log" 2>&1 || { echo "pmc pass $i ($ctrs) failed"; exit 1; }
done
"$PY" tools/pmc_sum.py "$OUT" "$KERNEL" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
