#!/usr/bin/env bash
# Interleaved A/B of encode tuning defines (tuning library): DEFS="a;b" (";"-separated, "-" = none).
set -u
export TMPDIR=/tmp MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so
mkdir -p gpurun_out
IFS=';' read -r -a L <<< "${DEFS:--}"
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CFGS:-C B}; do
    for d in "${L[@]}"; do
      dd=""; [ "$d" != "-" ] && dd="$d"
      MURR_JIT_DEFS="$dd" timeout -k 10 200 python bench.py --mode encode --enc-config $c --steps 10 --warmup 2 > gpurun_out/eab.json 2> gpurun_out/eab.err || { echo "FAIL $d"; tail -5 gpurun_out/eab.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1]);print('$c', '%-24s'%'$d', d['kernel_ms_avg'], d['frac_of_8TBs'], d['ms_per_step'])"
    done
  done
done
