#!/usr/bin/env bash
# Wide-schema (configs C and D) JIT decode shape sweep.
set -u
for cfg in C D; do
  echo "== config $cfg (default shape)"
  ARGS="--config $cfg" SHAPES="5x1" LDSB=65536 bash tools/jit_sweep.sh || exit $?
  ARGS="--config $cfg" SHAPES="2x1 2x2 3x1 3x2 4x1 9x1" LDSB=65536 bash tools/jit_sweep.sh || exit $?
  ARGS="--config $cfg" SHAPES="2x1 3x1" LDSB=32768 bash tools/jit_sweep.sh || exit $?
done
