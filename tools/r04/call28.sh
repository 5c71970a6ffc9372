#!/usr/bin/env bash
# round 4, call 28: the whole GPU suite on the final kernels, smoke, then the
# round profile again (both parts) for the profile lines
set -u
export TMPDIR=/tmp
PY=$(readlink -f "$(command -v python3)")
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1000 $PY -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t28.txt 2>&1 || { tail -40 $O/t28.txt; exit 1; }
tail -1 $O/t28.txt
timeout -k 10 180 $PY -c "import __graft_entry__ as g; g.smoke()" > $O/smoke28.txt 2>&1 || { tail $O/smoke28.txt; exit 1; }
tail -2 $O/smoke28.txt
R=r04 bash tools/round_profile.sh > $O/profile28.txt 2>&1 || { tail -20 $O/profile28.txt; exit 1; }
grep -E "exit=" $O/profile28.txt
