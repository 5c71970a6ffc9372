#!/usr/bin/env bash
# Decode ablations (make -C murr_amd/csrc ablate): kernel ms of the headline
# bench with parts of the work switched off (MURR_ABLATE in murr_decode.hip).
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-prod 1 2 4 7}; do
  lib=murr_amd/libmurr_codec.so; [ "$v" != prod ] && lib=murr_amd/libmurr_codec_abl$v.so
  MURR_LIB=$(pwd)/$lib timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu ${ARGS:-} \
    > gpurun_out/ab.log 2> gpurun_out/ab.err || { echo "variant $v failed"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.log'));print('ablate=$v', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s')"
done
