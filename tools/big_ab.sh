#!/bin/bash
# A/B of the wide per-wave conv tiles on the MWT shapes (EWVIT_CONV_BIG), one process per value
set -u
O=gpurun_out; mkdir -p $O
for b in ${VALUES:-0 10 11 12}; do
  EWVIT_CONV_BIG=$b timeout -k 10 200 python tools/conv_bench.py --only mwt --variants 1 --iters 10 > $O/cb_big$b.log 2>&1 || exit 1
  echo "== BIG=$b"; grep -v amdgpu.ids $O/cb_big$b.log
done
