#!/bin/bash
# MWT branch workgroup cap re-sweep on this build (EWVIT_MWT_GRID_CAP), interleaved rounds
set -o pipefail
O=gpurun_out; mkdir -p $O
for r in 1 2; do for v in 160 128 144 176 192; do
  EWVIT_MWT_GRID_CAP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/capsw_$v.log 2>&1 || exit 1
  echo "cap=$v $(tail -1 $O/capsw_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
