#!/usr/bin/env bash
# Round 6, call 3: prepared read with the gathered block's utf8 index, the
# speculative row-offset probe and the Arrow C export; XWIN A/B again.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c3}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 700 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_ingest.py tests/test_gpu_table.py tests/test_gpu_hstream.py tests/test_gpu_multigpu_read.py tests/test_gpu_bench_launch.py -m gpu -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
TL=$PWD/murr_amd/libmurr_codec_tuning.so
run ab 600 "$PY" tools/ab.py --reps 4 \
  --env x0=MURR_LIB=$TL --env x0=MURR_JIT_DEFS=MJ_XWIN=0 \
  --env x1=MURR_LIB=$TL --env x1=MURR_JIT_DEFS=MJ_XWIN=1 "x0::--extra-lanes 0" "x1::--extra-lanes 0"
cp -r gpurun_out/ab $out/ab
echo done
