#!/usr/bin/env bash
# round 4, call 5: timeline of the streaming host decode (kernel + memory-copy
# trace, no counters), to see which of H2D / decode / D2H overlap
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04/hstrace
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o h -- "$PY" bench.py --mode host --config B --blocks 40 --warmup 3 --steps 3 > $O/run.log 2>&1 || exit 1
ls -R $O | head -30
