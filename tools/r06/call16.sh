#!/usr/bin/env bash
# Round 6, call 16: config C's decode shape (tuning build, MURR_JIT_SHAPE):
# 3x1 (the default) against 4x1, 5x1 (more decode waves per tile) and 3x2
# (two chunks per wave), interleaved.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c16}
mkdir -p $out
TL=$PWD/murr_amd/libmurr_codec_tuning.so
rm -rf gpurun_out/ab
timeout -k 10 900 "$PY" tools/ab.py --reps 2 \
  --env s31=MURR_LIB=$TL --env s41=MURR_LIB=$TL --env s41=MURR_JIT_SHAPE=4x1 \
  --env s51=MURR_LIB=$TL --env s51=MURR_JIT_SHAPE=5x1 --env s32=MURR_LIB=$TL --env s32=MURR_JIT_SHAPE=3x2 \
  "s31::--config C --blocks 10 --extra-lanes 0" "s41::--config C --blocks 10 --extra-lanes 0" \
  "s51::--config C --blocks 10 --extra-lanes 0" "s32::--config C --blocks 10 --extra-lanes 0" > $out/abshape.log 2>&1
rc=$?
cp -r gpurun_out/ab $out/abshape
tail -6 $out/abshape.log
exit $rc
