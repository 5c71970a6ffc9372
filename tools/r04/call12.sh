#!/usr/bin/env bash
# round 4, call 12: streaming host decode -- wait time vs host time, depth
# sweep, kernel copies (fused) vs copy engines
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/hs12
timeout -k 10 300 $PY -u -m pytest tests/test_gpu_hstream.py -x -q --timeout 120 --timeout-method thread > $O/t12.txt 2>&1 || { tail -40 $O/t12.txt; exit 1; }
tail -1 $O/t12.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
for d in 2 3 4 6; do
  timeout -k 10 300 $PY bench.py --mode host --config B --depth $d --no-cpu > $O/hs12/fused_d$d.json 2> $O/hs12/fused_d$d.err || { tail $O/hs12/fused_d$d.err; exit 1; }
done
for d in 3 4; do
  MURR_LIB=$T MURR_HSTREAM_DMA=1 timeout -k 10 300 $PY bench.py --mode host --config B --depth $d --no-cpu > $O/hs12/dma_d$d.json 2> $O/hs12/dma_d$d.err || { tail $O/hs12/dma_d$d.err; exit 1; }
done
$PY - <<'PYEOF'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04/hs12/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("pinned_source", "pageable_source"):
        p = d[k]
        print(f.split("/")[-1], k[:6], p["GiB_s_host_to_host"], "ms", p["ms_per_batch"], "sub", p["host_submit_ms_per_batch"],
              "next", p["host_next_ms_per_batch"], "wait", p.get("host_wait_ms_per_batch"), "h2d", p["h2d_ms_per_batch"],
              "k", p["kernel_ms_per_batch"], "d2h", p["d2h_ms_per_batch"])
PYEOF
