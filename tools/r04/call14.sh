#!/usr/bin/env bash
# round 4, call 14: the whole GPU suite after the decode-wait split and the
# host stream's engine-H2D / kernel-D2H default; host benches B and C
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 $PY -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t14.txt 2>&1 || { tail -40 $O/t14.txt; exit 1; }
tail -1 $O/t14.txt
timeout -k 10 300 $PY bench.py --mode host --config B > $O/host_B7.json 2> $O/host_B7.err || { tail $O/host_B7.err; exit 1; }
timeout -k 10 300 $PY bench.py --mode host --config C --rows 1000 --blocks 2000 --warmup 50 > $O/host_C7.json 2> $O/host_C7.err || { tail $O/host_C7.err; exit 1; }
$PY - <<'PYEOF'
import json
for f in ("gpurun_out/r04/host_B7.json", "gpurun_out/r04/host_C7.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("pinned_source", "pageable_source"):
        p = d[k]
        print(f.split("/")[-1], k[:6], p["GiB_s_host_to_host"], "ms", p["ms_per_batch"], "sub", p["host_submit_ms_per_batch"],
              "next", p["host_next_ms_per_batch"], "wait", p.get("host_wait_ms_per_batch"), "h2d", p["h2d_ms_per_batch"],
              "k", p["kernel_ms_per_batch"], "d2h", p["d2h_ms_per_batch"])
    print("serial builder", d.get("builder_serial"))
PYEOF
