#!/usr/bin/env bash
# round 4, call 1: interpreter resolution (exec refusals), HBM ceiling probe,
# decode grid A/B (co-resident persistent grid vs one workgroup per virtual block)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
{ type -a python3; readlink -f "$(command -v python3)"; echo "PATH=$PATH"; } > gpurun_out/r04/python3.txt 2>&1
timeout -k 10 120 tools/ubench/ceiling 2048 > gpurun_out/r04/ceiling.txt 2>&1 || exit 1
timeout -k 10 900 python3 tools/ab.py --reps 2 \
  "D::--config D --steps 10 --warmup 2" \
  "D_g::--config D --steps 10 --warmup 2 --opts grid=-1" \
  "D_g_v1k::--config D --steps 10 --warmup 2 --opts grid=-1,vrows=1024" \
  "D_g_5x1::--config D --steps 10 --warmup 2 --opts grid=-1,shape=5x1" \
  "D_g_5x2::--config D --steps 10 --warmup 2 --opts grid=-1,shape=5x2" \
  "C::--config C --blocks 10 --steps 10 --warmup 2" \
  "C_g::--config C --blocks 10 --steps 10 --warmup 2 --opts grid=-1" \
  "B::--steps 20 --warmup 5" \
  "B_cut_g6k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=6144" \
  "B_cut_g3k::--steps 20 --warmup 5 --opts mode=cut,grid=-1,vrows=3072" \
  > gpurun_out/r04/ab1.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_hstream.py tests/test_gpu_scan.py tests/test_gpu_multigpu_read.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/t_hstream.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --mode host --config B > gpurun_out/r04/host_B.json 2> gpurun_out/r04/host_B.err || exit 1
timeout -k 10 300 python3 bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 > gpurun_out/r04/host_C.json 2> gpurun_out/r04/host_C.err || exit 1
