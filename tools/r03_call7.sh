#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py tests/test_gpu_fullsize.py tests/test_gpu_resident.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/t_enc.log 2>&1 || { tail -20 gpurun_out/r03/t_enc.log; exit 1; }
tail -1 gpurun_out/r03/t_enc.log
export MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  for c in C B E; do
    for t in "" 128 256 512; do
      env ${t:+MURR_ENC_TILE=$t} timeout -k 10 200 python bench.py --mode encode --enc-config $c --steps 10 --warmup 2 > gpurun_out/eab.json 2> gpurun_out/eab.err || { tail -5 gpurun_out/eab.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1]);print('$c tile=${t:-default}', d['kernel_ms_avg'], d['frac_of_8TBs'], d['ms_per_step'])"
    done
  done
done
