#!/usr/bin/env bash
# Round 6, call 15: call 14 (the fused gather indexes the read's block; A/B
# against MURR_READ_NOIDX=1) with the gather's look-back words loaded
# together; the whole GPU suite first.
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
out=gpurun_out/r06/${TAG:-c15}
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 3 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
run tests 1000 "$PY" -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
TL=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  run res_C_idx_$rep 300 env MURR_LIB=$TL "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
  run res_C_noidx_$rep 300 env MURR_LIB=$TL MURR_READ_NOIDX=1 "$PY" bench.py --mode resident --keys 1000 --steps 300 --warmup 30
done
for rep in 1 2; do run res_plain_$rep 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 300 --warmup 30 --ipc; done
run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
echo done
