#!/usr/bin/env bash
# Round 6, call 35: the index at load <= 1/3 (3 slots per key, the new
# default): the whole GPU suite, the resident lines (config C, read_plain,
# read_block at 100 M rows) and the driver's default bench line.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c35}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 1 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 1000 "$PY" -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run resident_1000_long 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run resident_read_plain 400 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --ipc
run resident_read_block 600 "$PY" bench.py --mode resident --table ref --rows 100000000 --keys 1000 --steps 200 --warmup 20
run bench 400 "$PY" bench.py
echo done
