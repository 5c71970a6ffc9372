#!/usr/bin/env bash
# round 4, call 20: D shard deal orders -- index order / runs of 8 per XCD
# round-robin / runs of 8 with pseudo-random XCD order; per-XCD timelines
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/tl20
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for x in 0 1 2; do E="$E --env D_x$x=MURR_LIB=$T --env D_x$x=MURR_XORDER=$x"; done
timeout -k 10 600 $PY tools/ab.py --reps 3 $E \
  "D_x0::--config D --steps 10 --warmup 2" "D_x1::--config D --steps 10 --warmup 2" "D_x2::--config D --steps 10 --warmup 2" \
  > $O/ab20.txt 2>&1 || { tail -20 $O/ab20.txt; exit 1; }
tail -4 $O/ab20.txt
for x in 0 1 2; do
  rm -f $O/tl20/dump_x$x.csv
  MURR_LIB=$T MURR_XORDER=$x MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 MURR_TIMELINE_DUMP=$O/tl20/dump_x$x.csv \
    timeout -k 10 200 $PY tools/timeline_d.py 1250000 "verbose=1" > $O/tl20/tl_x$x.log 2>&1 || { tail $O/tl20/tl_x$x.log; exit 1; }
  grep -E "^run|end   " $O/tl20/tl_x$x.log | tail -2
done
