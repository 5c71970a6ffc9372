#!/usr/bin/env bash
# Decode tile-shape / LDS-budget sweep on one MI355X: kernel ms and achieved
# GB/s of the headline bench per setting.  SHAPES: "NWxKC" list ("auto" = the
# host's choice); LDSB: per-workgroup LDS budgets; ARGS: extra bench.py args.
set -u
mkdir -p gpurun_out
for lds in ${LDSB:-40960}; do
for sh in ${SHAPES:-auto}; do
  if [ "$sh" = auto ]; then unset MURR_DECODE_SHAPE; else export MURR_DECODE_SHAPE=$sh; fi
  MURR_DECODE_LDS=$lds MURR_DECODE_VERBOSE=1 timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu ${ARGS:-} \
    > gpurun_out/sw.log 2> gpurun_out/sw.err || { echo "shape $sh lds $lds failed"; tail -5 gpurun_out/sw.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw.log'));print('shape=$sh lds=$lds', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s', d['value'], 'GiB/s')"
  tail -1 gpurun_out/sw.err
done; done
true
