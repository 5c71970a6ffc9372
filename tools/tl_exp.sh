export MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_DECODE_VERBOSE=1
run() { # name stride opts defs
  UIDX_STRIDE=$2 MURR_JIT_DEFS=$4 timeout -k 10 200 python tools/timeline_d.py 1250000 "$3" > gpurun_out/tlx_$1.log 2>&1 || { echo "fail $1"; tail -3 gpurun_out/tlx_$1.log; exit 1; }
  echo "== $1"; grep -E "^run|end   |first tile|duration" gpurun_out/tlx_$1.log | tail -4
}
run s512q0 512 "verbose=1" "MJ_TIMELINE=1,MJ_QUEUE=0"
run s128q0 128 "verbose=1,vrows=128" "MJ_TIMELINE=1,MJ_QUEUE=0"
run s128q1 128 "verbose=1,vrows=128" "MJ_TIMELINE=1,MJ_QUEUE=1"
run s128v256q1 128 "verbose=1,vrows=256" "MJ_TIMELINE=1,MJ_QUEUE=1"
run s512q1 512 "verbose=1" "MJ_TIMELINE=1,MJ_QUEUE=1"
