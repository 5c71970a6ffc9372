#!/usr/bin/env bash
# Round 6, call 26: the final tree's resident reads (as the round profile
# runs them), with the CPU baseline of a read and the host split.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c26}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 1 "$out/$name.log" | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
}
run resident_1000 300 "$PY" bench.py --mode resident --keys 1000 --steps 30 --warmup 5
run resident_1000_long 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run resident_read_plain 400 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --ipc
run resident_read_block 600 "$PY" bench.py --mode resident --table ref --rows 100000000 --keys 1000 --steps 200 --warmup 20
echo done
