#!/usr/bin/env bash
# Quick decode/encode timing sweep on one GPU (headline B, wide C / D shard,
# encode E/B/C); one line per run under gpurun_out/perf/.
set -u
export TMPDIR=/tmp
out=gpurun_out/perf
mkdir -p $out
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 200 python3 bench.py "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"kernel_ms_avg": [0-9.]*\|"frac": [0-9.]*\|"frac_of_8TBs": [0-9.]*\|"value": [0-9.]*' $out/$name.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
run B --steps 20 --warmup 3 --no-cpu
run C --config C --blocks 10 --steps 10 --warmup 2 --no-cpu
run D1 --config D --steps 10 --warmup 2 --no-cpu
run D125 --config D --rows 100000 --blocks 125 --steps 10 --warmup 2 --no-cpu
if [ -n "${ENC:-}" ]; then
  run encE --mode encode --steps 10 --warmup 2
  run encB --mode encode --enc-config B --steps 10 --warmup 2
  run encC --mode encode --enc-config C --steps 10 --warmup 2
fi
