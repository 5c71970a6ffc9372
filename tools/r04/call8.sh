#!/usr/bin/env bash
# round 4, call 8: the whole GPU suite with early slot release; A/B of it
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 $PY -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t8.txt 2>&1 || { tail -40 $O/t8.txt; exit 1; }
tail -2 $O/t8.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 900 $PY tools/ab.py --reps 2 \
  --env B_noer=MURR_LIB=$T --env B_noer=MURR_JIT_DEFS=MJ_ER=0 \
  --env C_noer=MURR_LIB=$T --env C_noer=MURR_JIT_DEFS=MJ_ER=0 \
  --env D_noer=MURR_LIB=$T --env D_noer=MURR_JIT_DEFS=MJ_ER=0 \
  "B::--steps 20 --warmup 5" "B_noer::--steps 20 --warmup 5" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" "C_noer::--config C --blocks 10 --steps 10 --warmup 2" \
  "D::--config D --steps 10 --warmup 2" "D_noer::--config D --steps 10 --warmup 2" \
  > $O/ab8.txt 2>&1
tail -8 $O/ab8.txt
timeout -k 10 120 tools/ubench/pcie > $O/pcie2.txt 2>&1 || exit 1
timeout -k 10 300 $PY bench.py --mode host --config B --depth 4 > $O/host_B5.json 2> $O/host_B5.err || exit 1
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 --depth 4 > $O/host_C5.json 2> $O/host_C5.err || exit 1
for b in 1 0; do
  MURR_LIB=$T MURR_DECODE_VERBOSE=1 MURR_JIT_DEFS=MJ_TIMELINE=1 UIDX_STRIDE=128 timeout -k 10 200 $PY tools/timeline_d.py 1250000 "verbose=1,balance=$((b==1 ? 1 : 0))" > $O/tl_bal$b.log 2>&1 || exit 1
done
grep -E "^run|end   |duration|first tile|xcc" $O/tl_bal*.log | head -60
