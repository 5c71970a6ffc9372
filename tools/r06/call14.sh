#!/usr/bin/env bash
# Round 6, call 14: the fused gather writes the gathered block's utf8 index
# from the table's per-row string bytes (murr_utf8_row_lengths) and the
# read's decode cuts the block (one pass) instead of split mode; A/B against
# MURR_READ_NOIDX=1 (tuning build).  Gather / read / resident / SST tests first.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c14}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_table.py \
  tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -x -q --timeout 200 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_idx_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_C_noidx_$rep 300 env MURR_LIB=$TL MURR_READ_NOIDX=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
done
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
echo done
