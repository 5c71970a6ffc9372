#!/usr/bin/env bash
# Round 6, call 23: config C's cache policies (tuning build, MURR_JIT_DEFS):
# every output store non-temporal (MJ_OUT_NT=2), validity words non-temporal
# (MJ_OUT_NT_VAL=1), 1-byte values plain (MJ_OUT_NT_W1=0), non-temporal blob
# DMA (MJ_BLOB_NT=1), against the layout's default, interleaved.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c23}
mkdir -p $out
TL=$PWD/murr_amd/libmurr_codec_tuning.so
rm -rf gpurun_out/ab
timeout -k 10 1000 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL \
  --env nt2=MURR_LIB=$TL --env nt2=MURR_JIT_DEFS=MJ_OUT_NT=2 \
  --env ntval=MURR_LIB=$TL --env ntval=MURR_JIT_DEFS=MJ_OUT_NT_VAL=1 \
  --env w1=MURR_LIB=$TL --env w1=MURR_JIT_DEFS=MJ_OUT_NT_W1=0 \
  --env blobnt=MURR_LIB=$TL --env blobnt=MURR_JIT_DEFS=MJ_BLOB_NT=1 \
  "base::--config C --blocks 10 --extra-lanes 0" "nt2::--config C --blocks 10 --extra-lanes 0" \
  "ntval::--config C --blocks 10 --extra-lanes 0" "w1::--config C --blocks 10 --extra-lanes 0" \
  "blobnt::--config C --blocks 10 --extra-lanes 0" > $out/abC.log 2>&1
rc=$?
cp -r gpurun_out/ab $out/abC
tail -7 $out/abC.log
exit $rc
