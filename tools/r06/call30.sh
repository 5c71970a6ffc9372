#!/usr/bin/env bash
# Round 6, call 30: where a prepared read's fused gather spends its time --
# gather_fused's phase clocks (tuning build, MURR_GATHER_STAMPS=1) and the
# host run's phases (MURR_READ_PHASES=1) for config C and read_plain at
# several key counts; the read-plan tests under the stamped build first.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c30}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; grep -E "gather stamps|read plan phases" "$out/$name.log" | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run tests 600 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 "$PY" -u -m pytest tests/test_gpu_read_plan.py -x -q --timeout 300 --timeout-method thread
for k in 1000 256 64; do
  run stamps_C_$k 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 MURR_READ_PHASES=1 "$PY" bench.py --mode resident --keys $k --steps 200 --warmup 20 --no-cpu
done
run stamps_plain_1000 300 env MURR_LIB=$TL MURR_GATHER_STAMPS=1 MURR_READ_PHASES=1 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --no-cpu
echo done
