#!/usr/bin/env bash
# A/B of JIT kernel sources (SRCS: files for MURR_JIT_SRC, "-" = the embedded
# source) on the headline bench in one box session, alternating, REPS times.
set -u
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
for f in ${SRCS:--}; do
  if [ "$f" = "-" ]; then unset MURR_JIT_SRC; else export MURR_JIT_SRC=$f; fi
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu ${ARGS:-} > gpurun_out/abs.log 2> gpurun_out/abs.err || { echo "src $f failed"; tail -5 gpurun_out/abs.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abs.log'));print('src=$f', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s')"
done; done
