#!/usr/bin/env bash
# Round 6, call 24: non-temporal blob DMA (MJ_BLOB_NT=1) and plain 1-byte
# value stores (MJ_OUT_NT_W1=0) on C, D (one shard) and B, interleaved.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c24}
mkdir -p $out
TL=$PWD/murr_amd/libmurr_codec_tuning.so
ab() {  # ab <name> <args>
  local name=$1; shift
  rm -rf gpurun_out/ab
  timeout -k 10 1000 "$PY" tools/ab.py --reps 3 \
    --env base=MURR_LIB=$TL \
    --env bnt=MURR_LIB=$TL --env bnt=MURR_JIT_DEFS=MJ_BLOB_NT=1 \
    --env bntw1=MURR_LIB=$TL --env "bntw1=MURR_JIT_DEFS=MJ_BLOB_NT=1,MJ_OUT_NT_W1=0" \
    "base::$*" "bnt::$*" "bntw1::$*" > $out/ab_$name.log 2>&1
  local rc=$?
  cp -r gpurun_out/ab $out/ab_$name
  echo "== $name rc=$rc"; tail -4 $out/ab_$name.log | cut -c1-110
  [ $rc -eq 0 ] || exit $rc
}
ab C --config C --blocks 10 --extra-lanes 0
ab D --config D --extra-lanes 0
ab B --extra-lanes 0
echo done
