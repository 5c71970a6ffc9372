#!/usr/bin/env bash
# One GPU-box session: smoke, GPU parity tests, a short bench, a rocprof
# kernel-trace summary.  Every GPU step has its own time limit; the script stops
# at the first step that crashed, aborted or timed out.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
# the resolved interpreter after `--` (rocprofv3 execs it; a `python3` on PATH may be a wrapper)
PY=$(readlink -f "$(command -v python3)")
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name exit=$rc"
    tail -n 5 "gpurun_out/$name.log"
    case $rc in 0|1) return 0 ;; *) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
lscpu > gpurun_out/lscpu.log 2>&1 || true
step smoke 180 "$PY" -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 "$PY" -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
step bench 380 "$PY" bench.py ${BENCH_ARGS:-}
if [ -n "${PROFILE:-}" ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o decode -- "$PY" bench.py --steps 5 --warmup 1 --no-cpu
fi
