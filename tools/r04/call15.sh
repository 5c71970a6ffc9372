#!/usr/bin/env bash
# round 4, call 15: round profile part 1 (the driver's command traced, B/C/D
# with their traffic passes); host stream check
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
mkdir -p gpurun_out/r04
timeout -k 10 200 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/t15.txt 2>&1 || { tail -30 gpurun_out/r04/t15.txt; exit 1; }
tail -1 gpurun_out/r04/t15.txt
R=r04 PART=1 bash tools/round_profile.sh || exit 1
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 --no-cpu > gpurun_out/r04/host_C8.json 2> gpurun_out/r04/host_C8.err || exit 1
$PY -c "
import json; d=json.loads(open('gpurun_out/r04/host_C8.json').read().strip().splitlines()[-1]); print({k: d[k]['GiB_s_host_to_host'] for k in ('pinned_source','pageable_source')})"
