#!/usr/bin/env bash
# Kernel-trace stats of the encode bench (config B and C column sets).
set -u
export TMPDIR=/tmp
# the resolved interpreter after `--` (rocprofv3 execs it; a `python3` on PATH may be a wrapper)
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/encprof
mkdir -p $out
for c in B C; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$c -o enc -- "$PY" bench.py --mode encode --enc-config $c --steps 10 --warmup 2 > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
  tail -1 $out/$c.log
  f=$(find $out/$c -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f"
done
