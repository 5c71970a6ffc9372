#!/usr/bin/env bash
# round 4, call 24: non-temporal output stores / blob loads on the D shard and
# C (the end-of-kernel writeback of dirty L2 lines), 4 workgroups per CU
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for v in D D_ont D_bnt D_both D_g1024 C C_ont; do E="$E --env $v=MURR_LIB=$T"; done
E="$E --env D_ont=MURR_JIT_DEFS=MJ_OUT_NT=1 --env D_bnt=MURR_JIT_DEFS=MJ_BLOB_NT=1 --env D_both=MURR_JIT_DEFS=MJ_OUT_NT=1,MJ_BLOB_NT=1 --env C_ont=MURR_JIT_DEFS=MJ_OUT_NT=1"
timeout -k 10 800 $PY tools/ab.py --reps 3 $E \
  "D::--config D --steps 10 --warmup 2" "D_ont::--config D --steps 10 --warmup 2" "D_bnt::--config D --steps 10 --warmup 2" \
  "D_both::--config D --steps 10 --warmup 2" "D_g1024::--config D --steps 10 --warmup 2 --opts grid=1024" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_ont::--config C --blocks 10 --steps 10 --warmup 2" \
  > $O/ab24.txt 2>&1 || { tail -20 $O/ab24.txt; exit 1; }
tail -8 $O/ab24.txt
