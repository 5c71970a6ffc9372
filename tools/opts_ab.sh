#!/usr/bin/env bash
# Interleaved A/B of decode kernel options (bench.py --opts) on one box:
# OPTS="a;b;c" (";"-separated, "-" = defaults), ARGS (bench arguments), REPS.
# Prints kernel ms, frac and the launch per run.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -r -a L <<< "${OPTS:--}"
for rep in $(seq 1 ${REPS:-2}); do
  for o in "${L[@]}"; do
    oa=(); [ "$o" != "-" ] && oa=(--opts "$o")
    timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu ${ARGS:-} "${oa[@]}" > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAIL $o"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);r=d['roofline'];print('%-40s'%'$o', r['kernel_ms_avg'], r['frac'], d['ms_per_step'], d['config'].get('launch'))"
  done
done
