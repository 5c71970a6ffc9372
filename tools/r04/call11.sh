#!/usr/bin/env bash
# round 4, call 11: streaming host decode with kernel copies (fused transfers);
# D's dynamic tail re-tested on the barrier ring with the fast-start prologue
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > $O/t11.txt 2>&1 || { tail -40 $O/t11.txt; exit 1; }
tail -2 $O/t11.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
timeout -k 10 300 $PY bench.py --mode host --config B --depth 4 > $O/host_B6.json 2> $O/host_B6.err || { tail $O/host_B6.err; exit 1; }
MURR_LIB=$T MURR_HSTREAM_DMA=1 timeout -k 10 300 $PY bench.py --mode host --config B --depth 4 --no-cpu > $O/host_B6dma.json 2> $O/host_B6dma.err || { tail $O/host_B6dma.err; exit 1; }
timeout -k 10 300 $PY bench.py --mode host --config B --depth 8 --no-cpu > $O/host_B6d8.json 2> $O/host_B6d8.err || { tail $O/host_B6d8.err; exit 1; }
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 --depth 4 > $O/host_C6.json 2> $O/host_C6.err || { tail $O/host_C6.err; exit 1; }
timeout -k 10 600 $PY tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" "D_dyn::--config D --steps 10 --warmup 2 --opts balance=2" \
  "D_dyn70::--config D --steps 10 --warmup 2 --opts balance=70" \
  > $O/ab11.txt 2>&1 || { tail -20 $O/ab11.txt; exit 1; }
tail -4 $O/ab11.txt
rm -rf $O/hstrace3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/hstrace3 -o h -- $PY bench.py --mode host --config B --depth 4 --blocks 60 --warmup 5 --no-cpu > $O/hstrace3.json 2> $O/hstrace3.err || { tail -5 $O/hstrace3.err; exit 1; }
