#!/usr/bin/env bash
# JIT decode shape sweep on one MI355X: kernel ms and achieved GB/s of the
# headline bench per MURR_JIT_SHAPE ("NWxR[xSLOTS[xSLACK]]"), LDS budget LDSB.
set -u
mkdir -p gpurun_out
for sh in ${SHAPES:-5x2 5x1 3x2 3x4 9x1 9x2}; do
  MURR_JIT_LDS=${LDSB:-65536} MURR_JIT_SHAPE=$sh MURR_DECODE_VERBOSE=1 timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu ${ARGS:-} \
    > gpurun_out/js.log 2> gpurun_out/js.err || { echo "shape $sh failed"; tail -5 gpurun_out/js.err; continue; }
  python3 -c "import json;d=json.load(open('gpurun_out/js.log'));print('shape=$sh', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s', d['value'], 'GiB/s')"
  tail -1 gpurun_out/js.err
done
true
