set -u
mkdir -p gpurun_out
for pj in 0 1 0,1; do
  timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu --proj $pj > gpurun_out/abl_$pj.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/abl_$pj.log'));print('$pj', d['roofline']['kernel_ms_avg'], d['roofline']['achieved'])"
done
