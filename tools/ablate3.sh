set -u
mkdir -p gpurun_out
for tb in ${TBS:-16384 32768}; do
for cfg in "0 0" "0,1 0" "0,1 4"; do
  set -- $cfg
  MURR_DECODE_TILE_BYTES=$tb MURR_DEBUG_DECODE=$2 timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu --proj $1 > gpurun_out/abl.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/abl.log'));print('tile=$tb proj=$1 dbg=$2', d['roofline']['kernel_ms_avg'], d['roofline']['achieved'])"
done; done
