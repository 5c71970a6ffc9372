#!/usr/bin/env bash
# Round 6, call 7: config C's decode split by ablation -- the loader alone
# (the ring's own ceiling for C's 3x1 tiles), no value / string stores, the
# full kernel -- and D10M; interleaved A/B on one box.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c7}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 6 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
rm -rf gpurun_out/ab
run abC 900 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL \
  --env lo=MURR_LIB=$TL --env lo=MURR_JIT_DEFS=MJ_ABL_LOADONLY=1 \
  --env nost=MURR_LIB=$TL --env nost=MURR_JIT_DEFS=MJ_ABL_NOSTR=1,MJ_ABL_NOFIX=1 \
  "base::--config C --blocks 10 --extra-lanes 0" "lo::--config C --blocks 10 --extra-lanes 0 --no-verify" \
  "nost::--config C --blocks 10 --extra-lanes 0 --no-verify"
cp -r gpurun_out/ab $out/abC
echo done
