#!/usr/bin/env bash
# Direct-load decode (every tile on the HBM-source path: stage 1 KiB) vs staged.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 100 python3 bench.py "$@" --no-cpu > gpurun_out/sd.log 2>&1 || { tail -3 gpurun_out/sd.log; exit 1; }
  echo "$name $(grep -o 'decode launch[^"]*' gpurun_out/sd.log | tail -1 | cut -c15-75) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/sd.log | tr '\n' ' ')"
}
run C_def X=1 -- --config C --blocks 10 --steps 10 --warmup 2
run C_direct MURR_JIT_STAGE=1024 -- --config C --blocks 10 --steps 10 --warmup 2
run C_direct_3x1 MURR_JIT_STAGE=1024 MURR_JIT_SHAPE=3x1 -- --config C --blocks 10 --steps 10 --warmup 2
run C_direct_pf MURR_JIT_STAGE=1024 MURR_JIT_DEFS=MJ_PREFETCH=1 -- --config C --blocks 10 --steps 10 --warmup 2
run B_def X=1 -- --steps 10 --warmup 2
run B_direct MURR_JIT_STAGE=1024 -- --steps 10 --warmup 2
