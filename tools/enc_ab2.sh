#!/usr/bin/env bash
# Encode A/B over (MURR_JIT_DEFS, MURR_ENC_GRID) pairs: VARS="defs@grid;..." ("-" = unset).
set -u
export TMPDIR=/tmp MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so
IFS=';' read -r -a L <<< "${VARS:--@-}"
for rep in $(seq 1 ${REPS:-2}); do
  for c in ${CFGS:-C B E}; do
    for v in "${L[@]}"; do
      d=${v%@*}; g=${v#*@}; [ "$d" = "-" ] && d=""; e=(); [ "$g" != "-" ] && e=(MURR_ENC_GRID=$g)
      env MURR_JIT_DEFS="$d" "${e[@]}" timeout -k 10 200 python bench.py --mode encode --enc-config $c --steps 10 --warmup 2 > gpurun_out/eab.json 2> gpurun_out/eab.err || { echo "FAIL $v"; tail -5 gpurun_out/eab.err; exit 1; }
      python3 -c "import json;d=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1]);print('$c', '%-24s'%'$v', d['kernel_ms_avg'], d['frac_of_8TBs'], d['ms_per_step'])"
    done
  done
done
