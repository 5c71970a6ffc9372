#!/usr/bin/env bash
# A/B of two library builds (LIBS: paths, "-" = the in-tree build) on the
# headline bench in one box session, alternating, REPS times.
set -u
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for l in ${LIBS:-- murr_amd/libmurr_codec_prev.so}; do
  if [ "$l" = "-" ]; then unset MURR_LIB; else export MURR_LIB=$l; fi
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu ${ARGS:-} > gpurun_out/abl.log 2> gpurun_out/abl.err || { echo "lib $l failed"; tail -5 gpurun_out/abl.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abl.log'));print('lib=$l', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s')"
done; done
