#!/usr/bin/env bash
# round 4, call 3: host link probe, streaming host bench v2 (shared copy
# streams, exact-size D2H), hstream parity, B decode over cut virtual blocks
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 120 tools/ubench/pcie > $O/pcie.txt 2>&1 || exit 1
timeout -k 10 300 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > $O/t_hstream2.txt 2>&1 || exit 1
timeout -k 10 300 $PY bench.py --mode host --config B > $O/host_B2.json 2> $O/host_B2.err || exit 1
timeout -k 10 300 $PY bench.py --mode host --config B --depth 4 > $O/host_B2d4.json 2> $O/host_B2d4.err || exit 1
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 > $O/host_C2.json 2> $O/host_C2.err || exit 1
timeout -k 10 900 $PY tools/ab.py --reps 2 \
  "B::--steps 20 --warmup 5" \
  "B_cut::--steps 20 --warmup 5 --opts mode=cut" \
  "B_cut_g6k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=6144" \
  "B_cut_g12k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=12288" \
  "B_cut_g24k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=24576" \
  "B_cut_g4k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=4096" \
  > $O/ab3.txt 2>&1
