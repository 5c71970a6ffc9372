#!/usr/bin/env bash
# Round 6, call 31: the final tree (after calls 29-30): the whole GPU suite and the driver's
# default bench line.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c31}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 1000 "$PY" -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench 400 "$PY" bench.py
echo done
