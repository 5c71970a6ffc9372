#!/usr/bin/env bash
# Headline config B: decode shape sweep (MURR_JIT_SHAPE), one line per run.
set -u
export TMPDIR=/tmp MURR_DECODE_VERBOSE=1
for sh in "" 5x2 9x1 9x2 5x1; do
  MURR_JIT_SHAPE=$sh timeout -k 10 100 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/sb.log 2>&1 || { tail -3 gpurun_out/sb.log; exit 1; }
  echo "B[$sh] $(grep -o 'decode launch[^"]*' gpurun_out/sb.log | tail -1 | cut -c1-120) | $(grep -o '"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/sb.log | tr '\n' ' ')"
done
