#!/usr/bin/env bash
# round 4, call 41: prepared plans timed one run in 1 / 4 / 8; the plan tests
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 300 $PY -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_plan.py tests/test_gpu_bench_launch.py > $O/t41.txt 2>&1 || { tail -30 $O/t41.txt; exit 1; }
tail -2 $O/t41.txt
E=""
for c in D B; do for v in 1 4 8; do E="$E --env ${c}_t$v=MURR_LIB=$T --env ${c}_t$v=MURR_TIME_EVERY=$v"; done; done
timeout -k 10 900 $PY tools/ab.py --reps 3 $E \
  "D_t1::--config D --steps 40 --warmup 3" "D_t4::--config D --steps 40 --warmup 3" "D_t8::--config D --steps 40 --warmup 3" \
  "B_t1::--steps 40 --warmup 5" "B_t4::--steps 40 --warmup 5" "B_t8::--steps 40 --warmup 5" \
  > $O/ab41.txt 2>&1 || { tail -20 $O/ab41.txt; exit 1; }
tail -7 $O/ab41.txt
