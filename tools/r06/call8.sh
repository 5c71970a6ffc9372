#!/usr/bin/env bash
# Round 6, call 8: the whole GPU suite on the current tree; prepared-read
# benches (config C, read_plain, read_block) and a trace; config C's decode
# split by ablation (loader alone / no value and string stores / full).
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c8}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 "$PY" -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
TL=$PWD/murr_amd/libmurr_codec_tuning.so
rm -rf gpurun_out/ab
run abC 900 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL \
  --env lo=MURR_LIB=$TL --env lo=MURR_JIT_DEFS=MJ_ABL_LOADONLY=1 \
  --env nost=MURR_LIB=$TL --env nost=MURR_JIT_DEFS=MJ_ABL_NOSTR=1,MJ_ABL_NOFIX=1 \
  --env ff=MURR_LIB=$TL --env ff=MURR_JIT_DEFS=MJ_FULLFAST=1 \
  "base::--config C --blocks 10 --extra-lanes 0" "lo::--config C --blocks 10 --extra-lanes 0 --no-verify" \
  "nost::--config C --blocks 10 --extra-lanes 0 --no-verify" "ff::--config C --blocks 10 --extra-lanes 0"
cp -r gpurun_out/ab $out/abC
rm -rf gpurun_out/ab
run abB 600 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL --env ff=MURR_LIB=$TL --env ff=MURR_JIT_DEFS=MJ_FULLFAST=1 \
  "base::--extra-lanes 0" "ff::--extra-lanes 0"
cp -r gpurun_out/ab $out/abB
echo done
