#!/usr/bin/env bash
# Round 6, call 10: split-mode segments claimed in run order when a launch
# has more segments than workgroups (seg_claim): the overlapped-split test
# first, then the whole GPU suite; config C without its index on 1 and 3
# lanes; the prepared reads (their one-round split launches keep the static
# deal); config C with its index (no split) as a control.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c10}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 4 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run t_overlap 300 "$PY" -u -m pytest tests/test_gpu_plan.py -k "overlapped or split" -x -q --timeout 200 --timeout-method thread
run tests 1000 "$PY" -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run C_noindex 300 "$PY" bench.py --config C --blocks 10 --steps 10 --warmup 2 --no-cpu --uidx-stride 0
run res_C 300 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
run res_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc
run C 300 "$PY" bench.py --config C --blocks 10 --steps 10 --warmup 2 --no-cpu
echo done
