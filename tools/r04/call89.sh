#!/usr/bin/env bash
set -u
bash tools/r04/call8.sh || exit 1
bash tools/r04/call9.sh
