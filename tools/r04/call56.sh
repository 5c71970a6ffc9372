#!/usr/bin/env bash
set -u
bash tools/r04/call5.sh > gpurun_out/r04_call5.log 2>&1 || { echo "call5 failed"; cat gpurun_out/r04_call5.log | tail -5; }
bash tools/r04/call6.sh
