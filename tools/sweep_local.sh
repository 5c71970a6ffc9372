#!/usr/bin/env bash
# Local-mode (one pass) vs split-mode decode of the config-C layout at equal bytes.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
out=gpurun_out/sweepL
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 100 python3 bench.py "$@" --no-cpu > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o 'decode launch[^"]*' $out/$name.log | tail -1 | cut -c1-150) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' $out/$name.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
run C1000x10k --config C --rows 10000 --blocks 1000 --steps 5 --warmup 1
run C2000x5k --config C --rows 5000 --blocks 2000 --steps 5 --warmup 1
run C500x20k --config C --rows 20000 --blocks 500 --steps 5 --warmup 1
MURR_JIT_MODE=split run C1000x10k_split --config C --rows 10000 --blocks 1000 --steps 5 --warmup 1
run C1000x10k_fixedonly --config C --rows 10000 --blocks 1000 --steps 5 --warmup 1 --proj 0,1,2,3,4,5,6,7,8,9,10,13,14,15
run C1000x10k_utf8only --config C --rows 10000 --blocks 1000 --steps 5 --warmup 1 --proj 11,12
