#!/usr/bin/env bash
# Decode shape sweep (MURR_JIT_SHAPE / MURR_JIT_LDS / MURR_JIT_SLACK): one line per run.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
run() {  # run <label> <env...> -- <bench args>
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 100 python3 bench.py "$@" --no-cpu > gpurun_out/sb.log 2>&1 || { tail -3 gpurun_out/sb.log; exit 1; }
  echo "$name $(grep -o 'decode launch[^"]*' gpurun_out/sb.log | tail -1 | cut -c15-130) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/sb.log | tr '\n' ' ')"
}
run B_def X=1 -- --steps 10 --warmup 2
run B_s3_40k MURR_JIT_SHAPE=5x2s3 MURR_JIT_LDS=40960 MURR_JIT_SLACK=1.08 -- --steps 10 --warmup 2
run B_s3_48k MURR_JIT_SHAPE=5x2s3 MURR_JIT_LDS=49152 -- --steps 10 --warmup 2
run B_5x1s3 MURR_JIT_SHAPE=5x1s3 MURR_JIT_LDS=26624 -- --steps 10 --warmup 2
run C_def X=1 -- --config C --blocks 10 --steps 5 --warmup 1
run C_5x1s3_96k MURR_JIT_SHAPE=5x1s3 MURR_JIT_LDS=98304 -- --config C --blocks 10 --steps 5 --warmup 1
run C_5x2_80k MURR_JIT_SHAPE=5x2 MURR_JIT_LDS=81920 -- --config C --blocks 10 --steps 5 --warmup 1
