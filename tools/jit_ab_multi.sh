#!/usr/bin/env bash
# A/B of JIT decode variants on several bench configs (CONFIGS:
# "name:args;name:args"), REPS times interleaved.  A variant is
# "DEFS" or "DEFS|ENV=V,ENV=V": DEFS goes to MURR_JIT_DEFS ("-" = none),
# the ENV assignments to the bench's environment.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra CFGS <<< "${CONFIGS:-B:}"
for rep in $(seq 1 ${REPS:-2}); do
for c in "${CFGS[@]}"; do
  name=${c%%:*}; args=${c#*:}
  for v in ${VARIANTS:--}; do
    d=${v%%|*}; e=""; [ "$d" != "$v" ] && e=${v#*|}
    [ "$d" = "-" ] && d=""
    envs=(); IFS=',' read -ra envs <<< "$e"
    env MURR_JIT_DEFS="$d" "${envs[@]}" timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu $args > gpurun_out/ab.log 2> gpurun_out/ab.err || { echo "$name variant $v failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.log'));r=d['roofline'];print('$name', 'variant=$v', round(r['kernel_ms_avg'],4), 'ms frac', r['frac'])"
  done
done; done
