#!/usr/bin/env bash
# Round 6, call 13: split mode's look-back over every utf8 column at once
# (MJ_LB_ALL=1, default) against one column at a time (MJ_LB_ALL=0), tuning
# build, interleaved: config C's prepared read and C without its index.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c13}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_decode.py tests/test_gpu_plan.py tests/test_gpu_read_plan.py -k "split or plan or read" -x -q --timeout 200 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_all_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_C_one_$rep 300 env MURR_LIB=$TL MURR_JIT_DEFS=MJ_LB_ALL=0 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
done
rm -rf gpurun_out/ab
run abCn 600 "$PY" tools/ab.py --reps 3 \
  --env all=MURR_LIB=$TL --env one=MURR_LIB=$TL --env one=MURR_JIT_DEFS=MJ_LB_ALL=0 \
  "all::--config C --blocks 10 --uidx-stride 0 --extra-lanes 0" "one::--config C --blocks 10 --uidx-stride 0 --extra-lanes 0"
cp -r gpurun_out/ab $out/abCn
echo done
