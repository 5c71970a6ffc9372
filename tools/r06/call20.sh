#!/usr/bin/env bash
# Round 6, call 20: resident reads with their CPU baseline (the oracle's
# MemoryStore restatement on one host thread) for config C and read_plain.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c20}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
run res_C 400 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 400 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
echo done
