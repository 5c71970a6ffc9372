#!/bin/bash
# SST count-kernel phase ablations (tuning library, MURR_SST_PROBE): kernel
# trace of bench.py --mode sst per probe value; summaries under $1.
set -e
out=${1:-gpurun_out/r05/sst_probe}
mkdir -p "$out"
PY=$(readlink -f "$(command -v python3)")
for p in 0 4 1 2; do
  MURR_LIB=$PWD/murr_amd/libmurr_codec_tuning.so MURR_SST_PROBE=$p timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o p$p -- "$PY" bench.py --mode sst --steps 5 --warmup 2 --no-cpu > "$out/p$p.log" 2>&1
done
