#!/usr/bin/env bash
# round 4, call 21: per-XCD timeline of config B (local mode, and cut)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/tl21
T=$PWD/murr_amd/libmurr_codec_tuning.so
for m in local cut; do
  rm -f $O/tl21/dump_$m.csv
  o="verbose=1"; [ $m = cut ] && o="verbose=1,mode=cut"
  MURR_LIB=$T MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 MURR_TIMELINE_DUMP=$O/tl21/dump_$m.csv \
    timeout -k 10 300 $PY tools/timeline_b.py 1000 "$o" > $O/tl21/tl_$m.log 2>&1 || { tail $O/tl21/tl_$m.log; exit 1; }
  grep -E "^run|end   |xcc|^decode" $O/tl21/tl_$m.log | tail -11
done
