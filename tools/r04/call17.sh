#!/usr/bin/env bash
# round 4, call 17: the D shard's per-workgroup spread vs SIMD placement:
# timelines with a per-workgroup dump (HW_ID), 5 vs 4 workgroups per CU
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/tl17
T=$PWD/murr_amd/libmurr_codec_tuning.so
for g in 0 1024; do
  rm -f $O/tl17/dump_g$g.csv
  MURR_LIB=$T MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 MURR_TIMELINE_DUMP=$O/tl17/dump_g$g.csv \
    timeout -k 10 200 $PY tools/timeline_d.py 1250000 "verbose=1,grid=$g" > $O/tl17/tl_g$g.log 2>&1 || { tail $O/tl17/tl_g$g.log; exit 1; }
  grep -E "^run|end   |duration|dur simd" $O/tl17/tl_g$g.log | tail -7
done
exit 0
timeout -k 10 600 $PY tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" "D_g1024::--config D --steps 10 --warmup 2 --opts grid=1024" \
  "D_g768::--config D --steps 10 --warmup 2 --opts grid=768" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_g1024::--config C --blocks 10 --steps 10 --warmup 2 --opts grid=1024" \
  > $O/ab17.txt 2>&1 || { tail -20 $O/ab17.txt; exit 1; }
tail -6 $O/ab17.txt
