#!/bin/bash
# configs 5 and 4 on the final build, then the PMC traffic passes for config 2
set -o pipefail
O=gpurun_out; mkdir -p $O
for c in 5 4; do
  timeout -k 10 400 python bench.py --config $c --steps 20 > $O/bench_c${c}_final.log 2>&1 || exit 1
  echo "config $c: $(tail -1 $O/bench_c${c}_final.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
bash tools/gpu_pmc.sh
