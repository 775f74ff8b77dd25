#!/bin/bash
# A/B: backbone wgrad pixel-split target (EWVIT_WSPLIT_WG), then the compile + dp-graph tests in one process
set -o pipefail
O=gpurun_out; mkdir -p $O
for r in 1 2; do for v in 512 256 128; do
  EWVIT_WSPLIT_WG=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab_ws$v.log 2>&1 || exit 1
  echo "WSPLIT_WG=$v $(tail -1 $O/ab_ws$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_custom_ops.py tests/test_gpu_dp_graph.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/dp_diag2.log 2>&1
rc=$?; echo "dp2 rc=$rc"; tail -2 $O/dp_diag2.log; exit $rc
