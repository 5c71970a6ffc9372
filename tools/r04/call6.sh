#!/usr/bin/env bash
# round 4, call 6: decode parity (cut blocks, scans, resident reads) with the
# per-XCD dynamic tail; D / C / B A/B of the balance modes
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 $PY -u -m pytest tests/test_gpu_scan.py tests/test_gpu_decode.py tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > $O/t_dyn.txt 2>&1 || { tail -30 $O/t_dyn.txt; exit 1; }
tail -2 $O/t_dyn.txt
timeout -k 10 900 $PY tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" \
  "D_static::--config D --steps 10 --warmup 2 --opts balance=1" \
  "D_b30::--config D --steps 10 --warmup 2 --opts balance=30" \
  "D_b70::--config D --steps 10 --warmup 2 --opts balance=70" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" \
  "C_static::--config C --blocks 10 --steps 10 --warmup 2 --opts balance=1" \
  "D10M::--config D --rows 10000000 --steps 10 --warmup 2" \
  "D10M_static::--config D --rows 10000000 --steps 10 --warmup 2 --opts balance=1" \
  > $O/ab6.txt 2>&1
tail -12 $O/ab6.txt
