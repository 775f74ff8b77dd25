#!/bin/bash
# A/B: MWT on its own stream with its conv grids capped (EWVIT_MWT_GRID_CAP)
set -u
O=gpurun_out; mkdir -p $O
for r in ${ROUNDS:-1 2}; do for c in ${CAPS:-0 128 192 256 512}; do
  EWVIT_BRANCH_STREAMS=1 EWVIT_MWT_GRID_CAP=$c timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/cap_$c.log 2>&1 || exit 1
  echo "streams=1 cap=$c $(tail -1 $O/cap_$c.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done; done
