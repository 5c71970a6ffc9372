#!/usr/bin/env bash
# Round 6, call 27: the index's slot cache (murr_index_cache_rows): the read
# and index tests, then prepared reads with the cache and without
# (MURR_INDEX_NOCACHE=1, tuning build), interleaved, and a trace of 100 reads.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c27}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_table.py \
  tests/test_gpu_shard.py tests/test_gpu_ipc.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -x -q --timeout 300 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_rc_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_C_norc_$rep 300 env MURR_LIB=$TL MURR_INDEX_NOCACHE=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_rc_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_norc_$rep 300 env MURR_LIB=$TL MURR_INDEX_NOCACHE=1 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
done
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5 --no-cpu
echo done
