#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/tests_full.log 2>&1 || { tail -30 gpurun_out/r03/tests_full.log; exit 1; }
tail -2 gpurun_out/r03/tests_full.log
C16=$(python3 -c "print(','.join(str(i) for i in range(16)))")
R16=$(python3 -c "print(','.join(str(i) for i in reversed(range(16))))")
for rep in 1 2; do
  for c in "B:" "B:--proj rev" "C:--config C --blocks 10" "C:--config C --blocks 10 --proj rev" "D:--config D" "D:--config D --proj rev"; do
    n=${c%%:*}; a=${c#*:}
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/ab.log 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$n', '${a:0:40}', r['kernel_ms_avg'], r['frac'], d['ms_per_step'])"
  done
done
CFGS="C" DEFS="-;MJE_PF=5;MJE_PF=7" bash tools/enc_ab.sh
