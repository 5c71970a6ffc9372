#!/usr/bin/env bash
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_table.py tests/test_gpu_resident.py tests/test_gpu_ingest.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/enc_tests.log 2>&1 || { tail -30 gpurun_out/r03/enc_tests.log; exit 1; }
tail -2 gpurun_out/r03/enc_tests.log
CFGS="C B E" DEFS="-;MJE_VBITS=0" bash tools/enc_ab.sh
