#!/usr/bin/env bash
# Decode shape / LDS-budget sweep on configs C and D1 (tuning knobs
# MURR_JIT_SHAPE, MURR_JIT_LDS, MURR_JIT_MODE); one line per run.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
out=gpurun_out/sweep
mkdir -p $out
run() {  # run <name> <env...> -- <bench args...>
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 100 python3 bench.py "$@" --no-cpu > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o 'decode launch[^"]*' $out/$name.log | tail -1 | cut -c1-160) | $(grep -o '"frac": [0-9.]*' $out/$name.log)"
  [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
for cfg in "D1:--config D --steps 10 --warmup 2" "C:--config C --blocks 10 --steps 5 --warmup 1"; do
  n=${cfg%%:*}; a=${cfg#*:}
  run ${n}_def X=1 -- $a
  run ${n}_5x1_96k MURR_JIT_SHAPE=5x1 MURR_JIT_LDS=98304 -- $a
  run ${n}_3x1_40k MURR_JIT_SHAPE=3x1 MURR_JIT_LDS=40960 -- $a
  run ${n}_3x1_32k MURR_JIT_SHAPE=3x1 MURR_JIT_LDS=32768 -- $a
  run ${n}_5x2_80k MURR_JIT_SHAPE=5x2 MURR_JIT_LDS=81920 -- $a
  run ${n}_local MURR_JIT_MODE=local -- $a
done
