#!/usr/bin/env bash
# Decode parity tests, then the quick perf sweep (one GPU call).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_projection.py tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dec_t.log 2>&1
rc=$?
tail -3 gpurun_out/dec_t.log
[ $rc -eq 0 ] || exit $rc
bash tools/perf_quick.sh
