#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/t_enc.log 2>&1 || { tail -20 gpurun_out/r03/t_enc.log; exit 1; }
tail -1 gpurun_out/r03/t_enc.log
VARS="-@-;-@3" CFGS="E C B" REPS=1 bash tools/enc_ab2.sh
export MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so
for rep in 1 2; do
  for c in "D:--config D" "C:--config C --blocks 10" "B:"; do
    for g in "" 1; do
      n=${c%%:*}; a=${c#*:}
      env ${g:+MURR_JIT_GRIDALL=1} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$n gridall=$g', r['kernel_ms_avg'], r['frac'], d['ms_per_step'], d['config']['launch'])"
    done
  done
done
