#!/usr/bin/env bash
# A/B of decode tile shapes in one box session: each word of SHAPES is
# "NWxR" (bench.py --opts shape=...) or "-" (default selection); EXTRA is
# appended to --opts (e.g. lds=163840).  Prints kernel ms per shape,
# interleaved, REPS times.
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for s in ${SHAPES:--}; do
  o="${EXTRA:-}"; [ "$s" = "-" ] || o="shape=$s${EXTRA:+,$EXTRA}"
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${o:+--opts $o} ${ARGS:-} > gpurun_out/ab.log 2> gpurun_out/ab.err || { echo "shape $s failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.log'));r=d['roofline'];print('shape=$s', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s frac', r['frac'])"
done; done
