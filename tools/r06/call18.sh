#!/usr/bin/env bash
# Round 6, call 18: read-plan tests (utf8 counts 1 / 3 / 4 through the
# gather's index, a plan closed by a write), then the resident benches with
# the host read split three ways (Python keys, Arrow keys, the library run).
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c18}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 "$PY" -u -m pytest tests/test_gpu_read_plan.py tests/test_gpu_resident.py -x -q --timeout 200 --timeout-method thread
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
echo done
