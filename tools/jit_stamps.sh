#!/usr/bin/env bash
# Phase stamps of the JIT decode (MURR_JIT_DEFS=MJ_STAMPS build of the kernel) for the
# headline bench, per MURR_JIT_SHAPE.
set -u
mkdir -p gpurun_out
for sh in ${SHAPES:-5x2}; do
  MURR_JIT_SHAPE=$sh MURR_JIT_DEFS=MJ_STAMPS MURR_DECODE_VERBOSE=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu ${ARGS:-} \
    > gpurun_out/st.log 2> gpurun_out/st.err || { echo "shape $sh failed"; tail -5 gpurun_out/st.err; exit 1; }
  echo "shape=$sh"; grep stamps gpurun_out/st.err | tail -1
done
