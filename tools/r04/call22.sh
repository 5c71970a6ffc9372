#!/usr/bin/env bash
# round 4, call 22: config B whole blocks (1000 workgroups) vs cut into
# virtual blocks over a full 4-per-CU grid (plan path, the bench's launch)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 700 $PY tools/ab.py --reps 3 \
  "B::--steps 20 --warmup 5" "B_cut::--steps 20 --warmup 5 --opts mode=cut" \
  "B_cut11k::--steps 20 --warmup 5 --opts mode=cut,vrows=11264" \
  "B_cut25k::--steps 20 --warmup 5 --opts mode=cut,vrows=25088" \
  > $O/ab22.txt 2>&1 || { tail -20 $O/ab22.txt; exit 1; }
tail -5 $O/ab22.txt
