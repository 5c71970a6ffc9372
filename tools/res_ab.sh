set -u
mkdir -p gpurun_out
for st in "" 64; do for k in 1000 10000; do MURR_JIT_SEGTILES=$st timeout -k 10 120 python bench.py --mode resident --keys $k --steps 40 --warmup 5 > gpurun_out/ab_$k.log 2>&1 || exit $?; echo "segtiles=$st $(tail -1 gpurun_out/ab_$k.log)"; done; done
