#!/usr/bin/env bash
# round 4, call 26: non-temporal output stores -- values and offsets (1),
# and strings + validity words too (2) -- on B, C, D shard, D at 10 M rows
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for c in B C D D10; do
  for v in 0 1 2; do E="$E --env ${c}_nt$v=MURR_LIB=$T --env ${c}_nt$v=MURR_JIT_DEFS=MJ_OUT_NT=$v"; done
done
timeout -k 10 1000 $PY tools/ab.py --reps 2 $E \
  "B_nt0::--steps 20 --warmup 5" "B_nt1::--steps 20 --warmup 5" "B_nt2::--steps 20 --warmup 5" \
  "C_nt0::--config C --blocks 10 --steps 10 --warmup 2" "C_nt1::--config C --blocks 10 --steps 10 --warmup 2" "C_nt2::--config C --blocks 10 --steps 10 --warmup 2" \
  "D_nt0::--config D --steps 10 --warmup 2" "D_nt1::--config D --steps 10 --warmup 2" "D_nt2::--config D --steps 10 --warmup 2" \
  "D10_nt0::--config D --rows 10000000 --steps 5 --warmup 1" "D10_nt1::--config D --rows 10000000 --steps 5 --warmup 1" "D10_nt2::--config D --rows 10000000 --steps 5 --warmup 1" \
  > $O/ab26.txt 2>&1 || { tail -20 $O/ab26.txt; exit 1; }
tail -13 $O/ab26.txt
