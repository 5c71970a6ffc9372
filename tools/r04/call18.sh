#!/usr/bin/env bash
# round 4, call 18: dynamic tail as a last resort (80-90 % dealt statically),
# claims spread over time instead of clustered
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/tl18
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 600 $PY tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" "D_b90::--config D --steps 10 --warmup 2 --opts balance=90" \
  "D_b80::--config D --steps 10 --warmup 2 --opts balance=80" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_b90::--config C --blocks 10 --steps 10 --warmup 2 --opts balance=90" \
  > $O/ab18.txt 2>&1 || { tail -20 $O/ab18.txt; exit 1; }
tail -6 $O/ab18.txt
for b in 1 90; do
  rm -f $O/tl18/dump_b$b.csv
  MURR_LIB=$T MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 MURR_TIMELINE_DUMP=$O/tl18/dump_b$b.csv \
    timeout -k 10 200 $PY tools/timeline_d.py 1250000 "verbose=1,balance=$b" > $O/tl18/tl_b$b.log 2>&1 || { tail $O/tl18/tl_b$b.log; exit 1; }
  grep -E "^run|end   |duration|^decode" $O/tl18/tl_b$b.log | tail -4
done
