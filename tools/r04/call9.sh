#!/usr/bin/env bash
# round 4, call 9: encode counters (config C and B column sets)
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
OUT=$O/pmc_encC KERNEL=murr_jit_encode ARGS="--mode encode --enc-config C --steps 3 --warmup 1" timeout -k 10 400 bash tools/pmc_passes.sh > $O/pmc_encC.log 2>&1 || { tail -5 $O/pmc_encC.log; exit 1; }
OUT=$O/pmc_encB KERNEL=murr_jit_encode ARGS="--mode encode --enc-config B --steps 3 --warmup 1" timeout -k 10 400 bash tools/pmc_passes.sh > $O/pmc_encB.log 2>&1 || { tail -5 $O/pmc_encB.log; exit 1; }
OUT=$O/pmc_B KERNEL=murr_jit_decode ARGS="--steps 3 --warmup 1" timeout -k 10 400 bash tools/pmc_passes.sh > $O/pmc_B.log 2>&1 || { tail -5 $O/pmc_B.log; exit 1; }
cat $O/pmc_encC/summary.txt $O/pmc_encB/summary.txt $O/pmc_B/summary.txt
