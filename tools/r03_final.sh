#!/usr/bin/env bash
# Round-3 closing call: full GPU suite, smoke, then the round profile.
set -u
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/tests_final.log 2>&1 || { tail -30 gpurun_out/r03/tests_final.log; exit 1; }
tail -2 gpurun_out/r03/tests_final.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
R=r03 bash tools/round_profile.sh
