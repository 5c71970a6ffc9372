#!/usr/bin/env bash
# round 4, call 4: store-shape probe; wide-layout (C) decode ablations
# (string stores / fixed-width stores skipped) with the tuning library
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 120 tools/ubench/stshape > $O/stshape.txt 2>&1 || exit 1
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 900 $PY tools/ab.py --reps 2 \
  --env C=MURR_LIB=$T --env C_nostr=MURR_LIB=$T --env C_nofix=MURR_LIB=$T --env C_none=MURR_LIB=$T \
  --env C_nostr=MURR_JIT_DEFS=MJ_ABL_NOSTR=1 --env C_nofix=MURR_JIT_DEFS=MJ_ABL_NOFIX=1 \
  --env C_none=MURR_JIT_DEFS=MJ_ABL_NOSTR=1,MJ_ABL_NOFIX=1 \
  "C::--config C --blocks 10 --steps 10 --warmup 2" \
  "C_nostr::--config C --blocks 10 --steps 10 --warmup 2 --no-verify" \
  "C_nofix::--config C --blocks 10 --steps 10 --warmup 2 --no-verify" \
  "C_none::--config C --blocks 10 --steps 10 --warmup 2 --no-verify" \
  > $O/ab4.txt 2>&1
timeout -k 10 300 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > $O/t_hstream3.txt 2>&1 || exit 1
timeout -k 10 300 $PY bench.py --mode host --config B > $O/host_B3.json 2> $O/host_B3.err || exit 1
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 > $O/host_C3.json 2> $O/host_C3.err || exit 1
