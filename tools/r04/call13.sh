#!/usr/bin/env bash
# round 4, call 13: PCIe concurrency of kernel and engine copies; streaming
# host decode variants (kernel copies both ways / engine H2D + kernel D2H /
# engine copies) and copy-kernel grids
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O/hs13
timeout -k 10 120 tools/ubench/pcie > $O/pcie3.txt 2>&1 || { tail $O/pcie3.txt; exit 1; }
grep concurrent $O/pcie3.txt
T=$PWD/murr_amd/libmurr_codec_tuning.so
run() {  # name, depth, env...
  local n=$1 d=$2; shift 2
  env MURR_LIB=$T "$@" timeout -k 10 300 $PY bench.py --mode host --config B --depth $d --no-cpu > $O/hs13/$n.json 2> $O/hs13/$n.err || { tail $O/hs13/$n.err; exit 1; }
}
run fused_d3 3 X=1
run hyb_d3 3 MURR_HSTREAM_H2D_ENGINE=1
run hyb_d4 4 MURR_HSTREAM_H2D_ENGINE=1
run fused_g16_d3 3 MURR_COPY_GRID_IN=16 MURR_COPY_GRID_OUT=32
run fused_g32_d4 4 MURR_COPY_GRID_IN=32 MURR_COPY_GRID_OUT=64
run dma_d3 3 MURR_HSTREAM_DMA=1
$PY - <<'PYEOF'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04/hs13/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    for k in ("pinned_source", "pageable_source"):
        p = d[k]
        print(f.split("/")[-1], k[:6], p["GiB_s_host_to_host"], "ms", p["ms_per_batch"], "sub", p["host_submit_ms_per_batch"],
              "next", p["host_next_ms_per_batch"], "wait", p.get("host_wait_ms_per_batch"), "h2d", p["h2d_ms_per_batch"],
              "k", p["kernel_ms_per_batch"], "d2h", p["d2h_ms_per_batch"])
PYEOF
