#!/usr/bin/env bash
# round 4, call 7: parity of the prefetched dynamic tail, the encode's string
# staging and the lighter host stream; A/B of each
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 $PY -u -m pytest tests/test_gpu_scan.py tests/test_gpu_decode.py tests/test_gpu_resident.py tests/test_gpu_encode.py tests/test_gpu_hstream.py tests/test_gpu_fullsize.py tests/test_gpu_table.py tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread > $O/t7.txt 2>&1 || { tail -30 $O/t7.txt; exit 1; }
tail -2 $O/t7.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 900 $PY tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" \
  "D_static::--config D --steps 10 --warmup 2 --opts balance=1" \
  "D_b30::--config D --steps 10 --warmup 2 --opts balance=30" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" \
  "C_static::--config C --blocks 10 --steps 10 --warmup 2 --opts balance=1" \
  > $O/ab7.txt 2>&1
tail -6 $O/ab7.txt
timeout -k 10 600 $PY tools/ab.py --reps 2 --env encC_off=MURR_LIB=$T --env encC_off=MURR_ENC_SBW=0 --env encB_off=MURR_LIB=$T --env encB_off=MURR_ENC_SBW=0 \
  "encC::--mode encode --enc-config C --steps 10 --warmup 2" \
  "encC_off::--mode encode --enc-config C --steps 10 --warmup 2" \
  "encB::--mode encode --enc-config B --steps 10 --warmup 2" \
  "encB_off::--mode encode --enc-config B --steps 10 --warmup 2" \
  "encE::--mode encode --enc-config E --steps 10 --warmup 2" \
  > $O/ab7e.txt 2>&1
tail -6 $O/ab7e.txt
timeout -k 10 300 $PY bench.py --mode host --config B > $O/host_B4.json 2> $O/host_B4.err || exit 1
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 > $O/host_C4.json 2> $O/host_C4.err || exit 1
