#!/usr/bin/env bash
# round 4, call 19: virtual blocks dealt in runs of 8 per XCD (output lines
# written from one L2) vs index order
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/tl19
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 400 $PY -u -m pytest tests/test_gpu_scan.py tests/test_gpu_decode.py -x -q -k "cut or scan or shard" --timeout 120 --timeout-method thread > $O/t19.txt 2>&1 || { tail -30 $O/t19.txt; exit 1; }
tail -1 $O/t19.txt
E="--env D=MURR_LIB=$T --env D_nox=MURR_LIB=$T --env D_nox=MURR_XORDER=0 --env C=MURR_LIB=$T --env C_nox=MURR_LIB=$T --env C_nox=MURR_XORDER=0 --env D10=MURR_LIB=$T --env D10_nox=MURR_LIB=$T --env D10_nox=MURR_XORDER=0"
timeout -k 10 600 $PY tools/ab.py --reps 2 $E \
  "D::--config D --steps 10 --warmup 2" "D_nox::--config D --steps 10 --warmup 2" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_nox::--config C --blocks 10 --steps 10 --warmup 2" \
  "D10::--config D --rows 10000000 --steps 5 --warmup 1" "D10_nox::--config D --rows 10000000 --steps 5 --warmup 1" \
  > $O/ab19.txt 2>&1 || { tail -20 $O/ab19.txt; exit 1; }
tail -7 $O/ab19.txt
for x in 1 0; do
  rm -f $O/tl19/dump_x$x.csv
  MURR_LIB=$T MURR_XORDER=$x MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 MURR_TIMELINE_DUMP=$O/tl19/dump_x$x.csv \
    timeout -k 10 200 $PY tools/timeline_d.py 1250000 "verbose=1" > $O/tl19/tl_x$x.log 2>&1 || { tail $O/tl19/tl_x$x.log; exit 1; }
  grep -E "^run|end   |duration" $O/tl19/tl_x$x.log | tail -3
done
