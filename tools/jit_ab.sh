#!/usr/bin/env bash
# A/B of JIT decode variants in one box session: each line of VARIANTS is a
# MURR_JIT_DEFS value ("-" = none); prints kernel ms per variant, twice.
set -u
# MURR_JIT_DEFS is read by the tuning build only
export MURR_LIB=${MURR_LIB:-murr_amd/libmurr_codec_tuning.so}
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:--}; do
  d=$v; [ "$d" = "-" ] && d=""
  MURR_JIT_DEFS=$d timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu ${ARGS:-} > gpurun_out/ab.log 2> gpurun_out/ab.err || { echo "variant $v failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.log'));print('variant=$v', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s')"
done; done
