#!/usr/bin/env bash
# Round 6, call 17: this box's HBM ceilings (tools/ubench/ceiling: read, copy,
# B's exact 4:1:3 stream mix) beside the headline B line and config C, so the
# kernels' fractions can be set against the ceilings of one box.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c17}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run B1 300 "$PY" bench.py --no-cpu --extra-lanes 0
run ceiling 300 ./tools/ubench/ceiling 2048
run B2 300 "$PY" bench.py --no-cpu --extra-lanes 0
run C 300 "$PY" bench.py --config C --blocks 10 --no-cpu --extra-lanes 0
echo done
