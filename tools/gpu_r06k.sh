#!/bin/bash
set -uo pipefail
for cfg in "8 16" "4 16" "8 8"; do
  timeout -k 10 120 python tools/gat_pipe_debug2.py $cfg || exit 1
done
