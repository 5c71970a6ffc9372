#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
( export MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_DECODE_VERBOSE=1
  MURR_JIT_DEFS=MJ_TIMELINE=1 timeout -k 10 200 python tools/timeline_d.py 1250000 "verbose=1" > gpurun_out/r03/timeline_D.log 2>&1 )
grep -E "^run|end |first tile|duration|start" gpurun_out/r03/timeline_D.log | tail -8
CFGS=C DEFS="-;MJE_WPE=5;MJE_STAGE=30720,MJE_WPE=5;MJE_PF=1;MJE_STAGE=30720,MJE_WPE=5,MJE_PF=1" bash tools/enc_ab.sh > gpurun_out/r03/enc_occ.txt 2>&1
cat gpurun_out/r03/enc_occ.txt
R=r03 QUICK=1 bash tools/round_profile.sh
