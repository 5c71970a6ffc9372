#!/usr/bin/env bash
# Round profile on one MI355X: rocprofv3 kernel-trace stats of the headline
# bench, FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never combined with
# trace domains), then the headline bench line with roofline.traffic filled,
# plus the side measurements DESIGN.md quotes.  Everything under gpurun_out/$R.
set -u
export TMPDIR=/tmp
# the resolved interpreter after `--` (rocprofv3 execs it; a `python3` on PATH may be a wrapper)
PY=$(readlink -f "$(command -v python3)")
R=${R:-r06f}
PART=${PART:-all}  # 1: the headline trace and B/C/D with traffic; 2: the side measurements; all: both
out=gpurun_out/$R
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"; tail -n 2 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
if [ "$PART" != 2 ]; then
# the driver's exact command (bench.py --gpus 1 --steps 20 --warmup 5), traced
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o decode -- "$PY" bench.py --gpus 1 --steps 20 --warmup 5 --no-traffic
run fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc -o fetch -- "$PY" bench.py --steps 3 --warmup 1 --no-cpu --no-traffic
run write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc -o write -- "$PY" bench.py --steps 3 --warmup 1 --no-cpu --no-traffic
run bench 400 "$PY" bench.py --gpus 1 --steps 20 --warmup 5 --pmc-csv "$out/pmc/fetch_counter_collection.csv,$out/pmc/write_counter_collection.csv"
# wide-schema decode (configs C / D one-shard) with their own traffic passes
for cfg in "C:--config C --blocks 10" "D1:--config D"; do
  n=${cfg%%:*}; a=${cfg#*:}
  run fetch_$n 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc -o fetch_$n -- "$PY" bench.py $a --steps 3 --warmup 1 --no-cpu --no-traffic
  run write_$n 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc -o write_$n -- "$PY" bench.py $a --steps 3 --warmup 1 --no-cpu --no-traffic
  run decode_$n 300 "$PY" bench.py $a --steps 10 --warmup 2 --no-cpu --pmc-csv "$out/pmc/fetch_${n}_counter_collection.csv,$out/pmc/write_${n}_counter_collection.csv"
done
fi
if [ "$PART" != 1 ]; then
  run host_B 300 "$PY" bench.py --mode host --config B
  run encode_E 300 "$PY" bench.py --mode encode --steps 10 --warmup 2
  run decode_C_noindex 300 "$PY" bench.py --config C --blocks 10 --steps 10 --warmup 2 --no-cpu --uidx-stride 0
  run decode_D10M 300 "$PY" bench.py --config D --rows 10000000 --steps 10 --warmup 2 --no-cpu
  run decode_D1_noindex 300 "$PY" bench.py --config D --steps 10 --warmup 2 --no-cpu --uidx-stride 0
  run decode_B_generic 300 "$PY" bench.py --steps 10 --warmup 2 --no-cpu --opts kernel=generic
  run host_C 300 "$PY" bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50
  run encode_B 300 "$PY" bench.py --mode encode --enc-config B --steps 10 --warmup 2
  run encode_C 300 "$PY" bench.py --mode encode --enc-config C --steps 10 --warmup 2
  run resident_1000 300 "$PY" bench.py --mode resident --keys 1000 --steps 30 --warmup 5
  run resident_read_plain 300 "$PY" bench.py --mode resident --table ref --rows 10000000 --keys 1000 --steps 200 --warmup 20 --ipc
  # kernel trace of 100 prepared config-C reads (probe+scan, gather copy, decode)
  run trace_res_C 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_res_C -o res -- "$PY" bench.py --mode resident --keys 1000 --steps 100 --warmup 5
  run resident_read_block 400 "$PY" bench.py --mode resident --table ref --rows 100000000 --keys 1000 --steps 200 --warmup 20
  # one-block config D at 2x / 4x the shard: fixed cost per launch (fit over rows)
  run decode_D1x2 300 "$PY" bench.py --config D --rows 2500000 --steps 10 --warmup 2 --no-cpu
  run decode_D1x4 300 "$PY" bench.py --config D --rows 5000000 --steps 10 --warmup 2 --no-cpu
  run encode_prof 300 bash tools/enc_prof.sh
  run sst 300 "$PY" bench.py --mode sst --steps 10 --warmup 3
  # configs[3] as written at N = 1 (the whole 10 M-row table on one rank)
  run decode_D_table10M 400 "$PY" bench.py --config D --table-rows 10000000 --steps 10 --warmup 2 --no-cpu
  # per-workgroup timeline of the D shard (tuning build)
  run timeline_D 200 env MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 \
    "$PY" tools/timeline_d.py 1250000
fi
