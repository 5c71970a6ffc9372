#!/usr/bin/env bash
# A/B of a tuning define (default MJ_QUEUE: local mode's virtual-block queue)
# on configs B, C (10 x 1 M) and the D shard, interleaved; kernel ms per line.
set -u
export TMPDIR=/tmp MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so
mkdir -p gpurun_out
A=${A:-MJ_QUEUE=0}; B=${B:-MJ_QUEUE=1}
for rep in 1 2; do
  for c in "B:" "C:--config C --blocks 10" "D:--config D"; do
    n=${c%%:*}; a=${c#*:}
    for d in "$A" "$B"; do
      MURR_JIT_DEFS=$d timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/q.json 2> gpurun_out/q.err || { tail -5 gpurun_out/q.err; exit 1; }
      python3 -c "import json,sys;d=json.loads(open('gpurun_out/q.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$n', '$d', r['kernel_ms_avg'], r['frac'], d['ms_per_step'], d['config']['launch'])"
    done
  done
done
