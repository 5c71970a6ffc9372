#!/usr/bin/env bash
# Round 6, call 2: the prepared resident read (murr_read_plan) -- parity tests,
# the resident benches, a kernel + copy trace of 100 reads; counter passes on
# config C's 3x1 decode.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c2}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_ingest.py tests/test_gpu_bench_launch.py -m gpu -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 200 --warmup 20
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --ipc
run trace_res_C 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES" \
            "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  run pmc_C_$i 150 rocprofv3 --pmc $ctrs --output-format csv -d $out/pmc_C -o pass$i -- \
    "$PY" bench.py --config C --blocks 10 --steps 3 --warmup 1 --no-cpu --no-traffic --extra-lanes 0 --uidx-stride 512
done
"$PY" tools/pmc_sum.py $out/pmc_C murr_jit_decode_3x1 > $out/pmc_C_summary.txt 2>&1 || true
cat $out/pmc_C_summary.txt
echo done
