#!/usr/bin/env bash
# Round 6, call 34: the resident index at >= 4 slots per key (load <= 1/4;
# MURR_INDEX_SPREAD=4, tuning build) against the default 2: prepared reads,
# interleaved, and the gather's phase clocks for both.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c34}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; grep -E "gather stamps, device" "$out/$name.log" | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run tests 600 env MURR_LIB=$TL MURR_INDEX_SPREAD=4 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
  run res_C_s4_$rep 300 env MURR_LIB=$TL MURR_INDEX_SPREAD=4 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_C_s2_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_s4_$rep 300 env MURR_LIB=$TL MURR_INDEX_SPREAD=4 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_s2_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
done
run stamps_C_s4 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 MURR_INDEX_SPREAD=4 "$PY" bench.py --mode resident --keys 1000 --steps 200 --warmup 20 --no-cpu
run stamps_C_s2 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 "$PY" bench.py --mode resident --keys 1000 --steps 200 --warmup 20 --no-cpu
echo done
