#!/usr/bin/env bash
# Round 6, call 9: the small gather spread over one wave per 64 queries with a
# per-workgroup scan in the copy (gather_probe_wide / gather_scan_copy): the
# gather tests, then the prepared-read benches and a trace of 100 reads.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c9}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_resident.py tests/test_gpu_read_plan.py tests/test_gpu_table.py \
  tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_multigpu_read.py -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run res_C_tune 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_C_local 300 env MURR_LIB=$TL MURR_JIT_MODE=local "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain_local 300 env MURR_LIB=$TL MURR_JIT_MODE=local "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
echo done
