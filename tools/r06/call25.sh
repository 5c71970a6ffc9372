#!/usr/bin/env bash
# Round 6, call 25: column groups (MURR_JIT_CG=1, tuning build: the 3 x 1
# tiles of wide layouts decoded by four waves, two per 64-row chunk, fixed /
# utf8 columns): decode / plan / resident tests under it, then C and the D
# shard against the 3 x 1 default, interleaved.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c25}
mkdir -p $out
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
run t_cg 900 env MURR_LIB=$TL MURR_JIT_CG=1 "$PY" -u -m pytest tests/test_gpu_decode.py tests/test_gpu_plan.py tests/test_gpu_resident.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread
ab() {  # ab <name> <args>
  local name=$1; shift
  rm -rf gpurun_out/ab
  timeout -k 10 900 "$PY" tools/ab.py --reps 3 \
    --env base=MURR_LIB=$TL --env cg=MURR_LIB=$TL --env cg=MURR_JIT_CG=1 \
    "base::$*" "cg::$*" > $out/ab_$name.log 2>&1
  local rc=$?
  cp -r gpurun_out/ab $out/ab_$name
  echo "== $name rc=$rc"; tail -3 $out/ab_$name.log | cut -c1-140
  [ $rc -eq 0 ] || exit $rc
}
ab C --config C --blocks 10 --extra-lanes 0
ab D --config D --extra-lanes 0
ab D10M --config D --rows 10000000 --extra-lanes 0
echo done
