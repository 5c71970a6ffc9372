set -u
mkdir -p gpurun_out
for tb in ${TBS:-16384 32768}; do
for cfg in ${CFGS:-"0,1:0" "0:0" "0,1:4" "0,1:8"}; do
  pj=${cfg%%:*}; dbg=${cfg##*:}
  lib=murr_amd/libmurr_codec.so; [ "$dbg" != 0 ] && lib=murr_amd/libmurr_codec_dbg.so
  MURR_LIB=$(pwd)/$lib MURR_DECODE_TILE_BYTES=$tb MURR_DEBUG_DECODE=$dbg timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu --proj $pj > gpurun_out/abl.log 2>gpurun_out/abl.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/abl.log'));print('tile=$tb proj=$pj dbg=$dbg', d['roofline']['kernel_ms_avg'], d['roofline']['achieved'])"
  if [ "$dbg" = 8 ]; then tail -1 gpurun_out/abl.err; fi
done; done
true
