#!/bin/bash
# A/B of two library builds (EWVIT_LIB=ab_lib/libewvit_old.so vs the in-tree one),
# interleaved rounds of the config-2 bench (box-to-box variance ~1.5 %: compare within one run)
set -u
O=gpurun_out; mkdir -p $O
for r in ${ROUNDS:-1 2 3}; do for v in old new; do
  if [ $v = old ]; then L=$PWD/ab_lib/libewvit_old.so; else L=; fi
  EWVIT_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 ${BENCH_ARGS:-} > $O/ab_$v.log 2>&1 || exit 1
  echo "round=$r lib=$v $(tail -1 $O/ab_$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done; done
