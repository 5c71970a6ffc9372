#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_plan.py tests/test_gpu_bench_launch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/tail_tests.log 2>&1 || { tail -30 gpurun_out/r03/tail_tests.log; exit 1; }
tail -2 gpurun_out/r03/tail_tests.log
( export MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_DECODE_VERBOSE=1
  for d in MJ_TIMELINE=1 MJ_TIMELINE=1,MJ_NOTAIL=1; do
    MURR_JIT_DEFS=$d timeout -k 10 200 python tools/timeline_d.py 1250000 "verbose=1" > gpurun_out/r03/tl_$d.log 2>&1
    echo "== $d"; grep -E "^decode|^run|end |first tile" gpurun_out/r03/tl_$d.log | tail -5
  done
  for d in MJ_TIMELINE=1 MJ_TIMELINE=1,MJ_NOTAIL=1; do
    UIDX_STRIDE=128 MURR_JIT_DEFS=$d timeout -k 10 200 python tools/timeline_d.py 1250000 "verbose=1,vrows=128" > gpurun_out/r03/tl128_$d.log 2>&1
    echo "== stride 128 $d"; grep -E "^decode|^run|end |first tile" gpurun_out/r03/tl128_$d.log | tail -5
  done )
for rep in 1 2; do
  for v in - MJ_NOTAIL=1; do
    d=$v; [ "$d" = "-" ] && d=""
    for c in "--config D" "--config C --blocks 10"; do
      MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_JIT_DEFS=$d timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $c > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', '$c', r['kernel_ms_avg'], r['frac'], d['ms_per_step'])"
    done
  done
done
for rep in 1 2; do
  for g in "" 4 8 16; do
    env MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so ${g:+MURR_ENC_GRID=$g} timeout -k 10 120 python bench.py --mode encode --enc-config C --steps 10 --warmup 2 > gpurun_out/eab.json 2> gpurun_out/eab.err || { tail -5 gpurun_out/eab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1]);print('enc C grid/CU=$g', d['kernel_ms_avg'], d['frac_of_8TBs'], d['ms_per_step'])"
  done
done
