set -u
for rep in 1 2 3; do
for v in "MURR_JIT_SHAPE=5x2x2" "MURR_JIT_RO8=1 MURR_JIT_SHAPE=5x2x2x1.25" "MURR_JIT_SHAPE=5x2x3"; do
  env $v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab.log 2> gpurun_out/ab.err || { echo "$v failed"; tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.log'));print('$v', d['roofline']['kernel_ms_avg'], 'ms', d['roofline']['achieved'], 'GB/s')"
done; done
timeout -k 10 120 ./tools/ubench/mix_bw
