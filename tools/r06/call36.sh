#!/usr/bin/env bash
# Round 6, call 36: the driver's default bench line twice on another box
# (the decode kernel is call 31's; call 35's box ran slow).
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c36}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 1 "$out/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
}
run bench_1 400 "$PY" bench.py
run bench_2 400 "$PY" bench.py
echo done
