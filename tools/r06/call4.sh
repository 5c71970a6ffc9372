#!/usr/bin/env bash
# Round 6, call 4: where a prepared read's time goes (phase clocks, with and
# without the gathered block's utf8 index, with and without the event sync
# after the kernel's done flag); the host stream's submit phases; the PCIe
# stream probe with two batches per engine copy.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c4}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_base_$rep 200 env MURR_LIB=$TL MURR_READ_PHASES=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_noix_$rep 200 env MURR_LIB=$TL MURR_READ_PHASES=1 MURR_READ_NOIX=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_nosync_$rep 200 env MURR_LIB=$TL MURR_READ_PHASES=1 MURR_PLAN_NOSYNC=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_noix_nosync_$rep 200 env MURR_LIB=$TL MURR_READ_PHASES=1 MURR_READ_NOIX=1 MURR_PLAN_NOSYNC=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
done
run host_B 300 env MURR_LIB=$TL MURR_HSTREAM_PHASES=1 "$PY" bench.py --mode host --config B
run pcie 300 tools/ubench/pcie
echo done
