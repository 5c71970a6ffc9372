#!/usr/bin/env bash
# Headline B: workgroups per CU (forced through the LDS stage size), whole
# blocks vs virtual blocks.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 100 python3 bench.py "$@" --no-cpu > gpurun_out/sw.log 2>&1 || { tail -3 gpurun_out/sw.log; exit 1; }
  echo "$name $(grep -o 'decode launch[^"]*' gpurun_out/sw.log | tail -1 | cut -c15-75) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/sw.log | tr '\n' ' ')"
}
run B_whole X=1 -- --steps 20 --warmup 3
for st in 16384 20480 32768; do
  run B_whole_st$st MURR_JIT_STAGE=$st -- --steps 20 --warmup 3
  run B_cut_st$st MURR_JIT_CUT=1 MURR_JIT_STAGE=$st -- --steps 20 --warmup 3
done
run C_def X=1 -- --config C --blocks 10 --steps 10 --warmup 2
run C_st40k MURR_JIT_STAGE=40960 -- --config C --blocks 10 --steps 10 --warmup 2
run C_5x2 MURR_JIT_SHAPE=5x2 MURR_JIT_STAGE=57344 -- --config C --blocks 10 --steps 10 --warmup 2
