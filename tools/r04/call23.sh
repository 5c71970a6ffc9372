#!/usr/bin/env bash
# round 4, call 23: encode tiles in runs per XCD (MJE_XRUN); decode run
# length of the D shard's XCD runs (MURR_XRUN)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 $PY -u -m pytest tests/test_gpu_encode.py -x -q --timeout 120 --timeout-method thread > $O/t23.txt 2>&1 || { tail -30 $O/t23.txt; exit 1; }
tail -1 $O/t23.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
E=""
for v in encB encC encE; do
  for r in 1 8 32; do E="$E --env ${v}_r$r=MURR_LIB=$T --env ${v}_r$r=MURR_JIT_DEFS=MJE_XRUN=$r"; done
done
for r in 8 16 64; do E="$E --env D_r$r=MURR_LIB=$T --env D_r$r=MURR_XRUN=$r"; done
timeout -k 10 800 $PY tools/ab.py --reps 2 $E \
  "encB_r1::--mode encode --enc-config B --steps 10 --warmup 2" "encB_r8::--mode encode --enc-config B --steps 10 --warmup 2" "encB_r32::--mode encode --enc-config B --steps 10 --warmup 2" \
  "encC_r1::--mode encode --enc-config C --steps 10 --warmup 2" "encC_r8::--mode encode --enc-config C --steps 10 --warmup 2" "encC_r32::--mode encode --enc-config C --steps 10 --warmup 2" \
  "encE_r1::--mode encode --enc-config E --steps 10 --warmup 2" "encE_r8::--mode encode --enc-config E --steps 10 --warmup 2" \
  "D_r8::--config D --steps 10 --warmup 2" "D_r16::--config D --steps 10 --warmup 2" "D_r64::--config D --steps 10 --warmup 2" \
  > $O/ab23.txt 2>&1 || { tail -20 $O/ab23.txt; exit 1; }
tail -12 $O/ab23.txt
