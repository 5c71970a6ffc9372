#!/usr/bin/env bash
# Round 6, call 19: 16-B value stores gathered by DPP (MJ_X4=1, tuning build)
# against the per-lane stores, on B and C, interleaved; the decode tests under
# MJ_X4=1 first; the gather tests after the two-launch form's removal.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c19}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run t_gather 600 "$PY" -u -m pytest tests/test_gpu_resident.py tests/test_gpu_read_plan.py -x -q --timeout 200 --timeout-method thread
run t_x4 900 env MURR_LIB=$TL MURR_JIT_DEFS=MJ_X4=1 "$PY" -u -m pytest tests/test_gpu_decode.py tests/test_gpu_plan.py -x -q --timeout 200 --timeout-method thread
rm -rf gpurun_out/ab
run abB 900 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL --env x4=MURR_LIB=$TL --env x4=MURR_JIT_DEFS=MJ_X4=1 \
  "base::--extra-lanes 0" "x4::--extra-lanes 0"
cp -r gpurun_out/ab $out/abB
rm -rf gpurun_out/ab
run abC 900 "$PY" tools/ab.py --reps 3 \
  --env base=MURR_LIB=$TL --env x4=MURR_LIB=$TL --env x4=MURR_JIT_DEFS=MJ_X4=1 \
  "base::--config C --blocks 10 --extra-lanes 0" "x4::--config C --blocks 10 --extra-lanes 0"
cp -r gpurun_out/ab $out/abC
echo done
