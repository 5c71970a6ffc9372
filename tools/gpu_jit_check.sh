#!/usr/bin/env bash
# One GPU-box pass over the run-time specialised decode: decode/table/full-size
# parity tests with the JIT kernel forced, then a tile-shape sweep of the
# headline bench.  Stops at the first step that crashed or timed out.
set -u
mkdir -p gpurun_out
MURR_DECODE_JIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_table.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_jit.log 2>&1; rc=$?; echo "jit tests rc=$rc"; tail -4 gpurun_out/t_jit.log
[ $rc -le 1 ] || exit $rc
bash tools/jit_sweep.sh
