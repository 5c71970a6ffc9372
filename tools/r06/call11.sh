#!/usr/bin/env bash
# Round 6, call 11: small gathers fused into one launch (gather_fused: probe,
# look-back over 64-query groups, copy) against the two-launch form
# (MURR_GATHER_TWO=1, tuning build); gather / read tests first.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c11}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_resident.py tests/test_gpu_read_plan.py tests/test_gpu_table.py \
  tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -x -q --timeout 200 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_fused_$rep 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_C_two_$rep 300 env MURR_LIB=$TL MURR_GATHER_TWO=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_plain_fused_$rep 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
  run res_plain_two_$rep 300 env MURR_LIB=$TL MURR_GATHER_TWO=1 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
done
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
echo done
