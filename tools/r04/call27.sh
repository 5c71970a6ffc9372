#!/usr/bin/env bash
# round 4, call 27: per-layout non-temporal value stores (release default now)
# checked on B/C/D; non-temporal blob stores in the encode (tuning)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 $PY -u -m pytest tests/test_gpu_decode.py tests/test_gpu_scan.py tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread > $O/t27.txt 2>&1 || { tail -30 $O/t27.txt; exit 1; }
tail -1 $O/t27.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for c in encB encC encE; do E="$E --env ${c}_nt=MURR_LIB=$T --env ${c}_nt=MURR_JIT_DEFS=MJE_OUT_NT=1 --env ${c}=MURR_LIB=$T"; done
timeout -k 10 1000 $PY tools/ab.py --reps 2 $E \
  "B::--steps 20 --warmup 5" "C::--config C --blocks 10 --steps 10 --warmup 2" "D::--config D --steps 10 --warmup 2" \
  "encB::--mode encode --enc-config B --steps 10 --warmup 2" "encB_nt::--mode encode --enc-config B --steps 10 --warmup 2" \
  "encC::--mode encode --enc-config C --steps 10 --warmup 2" "encC_nt::--mode encode --enc-config C --steps 10 --warmup 2" \
  "encE::--mode encode --enc-config E --steps 10 --warmup 2" "encE_nt::--mode encode --enc-config E --steps 10 --warmup 2" \
  > $O/ab27.txt 2>&1 || { tail -20 $O/ab27.txt; exit 1; }
tail -10 $O/ab27.txt
