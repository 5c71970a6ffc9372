#!/usr/bin/env bash
# Round 6, call 29: host reads stage keys as 32-B {length, key} records (one
# probe round trip for the key over PCIe): the read tests, then host reads
# with records and without (MURR_READ_NOREC=1, tuning build), interleaved,
# then the final tree's resident lines (as call 26 ran them).
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c29}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
run tests 900 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py tests/test_gpu_table.py \
  tests/test_gpu_ipc.py tests/test_gpu_shard.py tests/test_gpu_multigpu_read.py tests/test_gpu_sst.py -x -q --timeout 300 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_rec_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_C_norec_$rep 300 env MURR_LIB=$TL MURR_READ_NOREC=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_rec_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
  run res_plain_norec_$rep 300 env MURR_LIB=$TL MURR_READ_NOREC=1 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --no-cpu
done
run resident_1000 300 "$PY" bench.py --mode resident --keys 1000 --steps 30 --warmup 5
run resident_1000_long 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run resident_read_plain 400 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --ipc
run resident_read_block 600 "$PY" bench.py --mode resident --table ref --rows 100000000 --keys 1000 --steps 200 --warmup 20
echo done
