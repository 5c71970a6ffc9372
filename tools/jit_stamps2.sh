#!/usr/bin/env bash
# Phase stamps (MJ_STAMPS build) for B, C, D1: one verbose step each; then
# MJ_PREFETCH A/B.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in "B:" "C:--config C --blocks 10" "D1:--config D"; do
  n=${c%%:*}; a=${c#*:}
  MURR_JIT_DEFS=MJ_STAMPS=1 MURR_DECODE_VERBOSE=1 timeout -k 10 150 python bench.py --steps 1 --warmup 1 --no-cpu $a > gpurun_out/st_$n.log 2> gpurun_out/st_$n.err || { tail -5 gpurun_out/st_$n.err; exit 1; }
  echo "== $n"; grep -E "stamps|decode launch" gpurun_out/st_$n.err | tail -3
done
