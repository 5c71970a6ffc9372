#!/usr/bin/env bash
# round 4, call 25: host stream with parallel staging copies (pageable
# sources); non-temporal options on the D shard and C (call 24)
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > $O/t25.txt 2>&1 || { tail -30 $O/t25.txt; exit 1; }
tail -1 $O/t25.txt
timeout -k 10 300 $PY bench.py --mode host --config B --no-cpu > $O/host_B9.json 2> $O/host_B9.err || { tail $O/host_B9.err; exit 1; }
$PY -c "
import json; d=json.loads(open('$O/host_B9.json').read().strip().splitlines()[-1])
for k in ('pinned_source','pageable_source'): p=d[k]; print(k, p['GiB_s_host_to_host'], 'sub', p['host_submit_ms_per_batch'], 'wait', p['host_wait_ms_per_batch'])"
bash tools/r04/call24.sh
