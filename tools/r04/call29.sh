#!/usr/bin/env bash
# round 4, call 29: encode column descriptors from a lane table (MJE_TAB)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 $PY -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > $O/t29.txt 2>&1 || { tail -30 $O/t29.txt; exit 1; }
tail -1 $O/t29.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for c in encB encC encE; do E="$E --env ${c}=MURR_LIB=$T --env ${c}_old=MURR_LIB=$T --env ${c}_old=MURR_JIT_DEFS=MJE_TAB=0"; done
timeout -k 10 800 $PY tools/ab.py --reps 3 $E \
  "encB::--mode encode --enc-config B --steps 10 --warmup 2" "encB_old::--mode encode --enc-config B --steps 10 --warmup 2" \
  "encC::--mode encode --enc-config C --steps 10 --warmup 2" "encC_old::--mode encode --enc-config C --steps 10 --warmup 2" \
  "encE::--mode encode --enc-config E --steps 10 --warmup 2" "encE_old::--mode encode --enc-config E --steps 10 --warmup 2" \
  > $O/ab29.txt 2>&1 || { tail -20 $O/ab29.txt; exit 1; }
tail -7 $O/ab29.txt
