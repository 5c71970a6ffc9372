#!/usr/bin/env bash
# Round 6, call 5: the one-workgroup gather (probe + scan + utf8 index + copy)
# and the flag-only wait in prepared reads; the LDS-DMA vs register-staging
# load probe; the host stream's steady-state submit phases.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c5}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run tests 700 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_ingest.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -m gpu -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
run ldsdma 200 tools/ubench/ldsdma
run host_B 300 env MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_HSTREAM_PHASES=1 "$PY" bench.py --mode host --config B
echo done
