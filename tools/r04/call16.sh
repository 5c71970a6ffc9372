#!/usr/bin/env bash
# round 4, call 16: round profile part 2 (side measurements DESIGN.md quotes)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
R=r04 PART=2 bash tools/round_profile.sh
