#!/usr/bin/env bash
# Round 6, call 32: the slot-cache probe loads four consecutive slots per
# round trip (kProbeWindow) instead of one: the read / index tests, then
# prepared reads with the window and without (MURR_PROBE_W=1, tuning build),
# interleaved, and the gather's phase clocks for both.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c32}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; grep -E "gather stamps, device" "$out/$name.log" | cut -c1-260; tail -n 1 "$out/$name.log" | cut -c1-120
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_table.py \
  tests/test_gpu_ipc.py tests/test_gpu_shard.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -x -q --timeout 300 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_w4_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_C_w1_$rep 300 env MURR_LIB=$TL MURR_PROBE_W=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_w4_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_w1_$rep 300 env MURR_LIB=$TL MURR_PROBE_W=1 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
done
run stamps_C_w4 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 "$PY" bench.py --mode resident --keys 1000 --steps 200 --warmup 20 --no-cpu
run stamps_C_w1 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 MURR_PROBE_W=1 "$PY" bench.py --mode resident --keys 1000 --steps 200 --warmup 20 --no-cpu
echo done
