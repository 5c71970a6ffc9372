#!/usr/bin/env bash
# round 4, call 10: fast-start loader prologue (GPU suite, A/B, D timeline),
# static deal by default; a copy/kernel trace of the streaming host decode
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 $PY -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t10.txt 2>&1 || { tail -40 $O/t10.txt; exit 1; }
tail -2 $O/t10.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for c in B C D; do E="$E --env $c=MURR_LIB=$T --env ${c}_nofast=MURR_LIB=$T --env ${c}_nofast=MURR_JIT_DEFS=MJ_FASTSTART=0"; done
timeout -k 10 900 $PY tools/ab.py --reps 3 $E \
  "B::--steps 20 --warmup 5" "B_nofast::--steps 20 --warmup 5" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_nofast::--config C --blocks 10 --steps 10 --warmup 2" \
  "D::--config D --steps 10 --warmup 2" "D_nofast::--config D --steps 10 --warmup 2" \
  > $O/ab10.txt 2>&1 || { tail -20 $O/ab10.txt; exit 1; }
tail -8 $O/ab10.txt
for f in 1 0; do
  MURR_LIB=$T MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS="MJ_TIMELINE=1,MJ_FASTSTART=$f" timeout -k 10 200 $PY tools/timeline_d.py 1250000 > $O/tl_fast$f.log 2>&1 || exit 1
done
grep -E "^run|end   |duration|first tile" $O/tl_fast*.log | head -40
rm -rf $O/hstrace2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/hstrace2 -o h -- $PY bench.py --mode host --config B --depth 4 --blocks 60 --warmup 5 > $O/hstrace2.json 2> $O/hstrace2.err || { tail -5 $O/hstrace2.err; exit 1; }
find $O/hstrace2 -name "*.csv" | head
