#!/usr/bin/env bash
# Headline B: whole blocks (local) vs virtual blocks (MURR_JIT_CUT), a few V sizes.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 100 python3 bench.py "$@" --no-cpu > gpurun_out/sc.log 2>&1 || { tail -3 gpurun_out/sc.log; exit 1; }
  echo "$name $(grep -o 'decode launch[^"]*' gpurun_out/sc.log | tail -1 | cut -c15-110) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/sc.log | tr '\n' ' ')"
}
for rep in 1 2; do
run B_whole X=1 -- --steps 20 --warmup 3
run B_cut MURR_JIT_CUT=1 -- --steps 20 --warmup 3
run B_cut_50k MURR_JIT_CUT=1 MURR_JIT_VROWS=50176 -- --steps 20 --warmup 3
run B_cut_20k MURR_JIT_CUT=1 MURR_JIT_VROWS=20480 -- --steps 20 --warmup 3
done
