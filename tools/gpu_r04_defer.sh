#!/bin/bash
# deferred multi-use gradient sums (ewvit.grads.give): the GPU tests that exercise parameter
# gradients (config-5 chunks, graphs, DDP buckets, modules, layer-by-layer), then config 5 and 2 benches
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_graph.py tests/test_gpu_dp_graph.py tests/test_gpu_se.py tests/test_gpu_bn.py tests/test_gpu_modules.py tests/test_gpu_vit.py tests/test_gpu_head.py tests/test_gpu_hfsep.py tests/test_gpu_custom_ops.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/defer_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/defer_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 5 2; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --no-cpu-baseline > $O/defer_c$c.log 2>&1 || exit 1
  echo "config $c: $(tail -1 $O/defer_c$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
