#!/bin/bash
# BASELINE configs 4 and 5 on this build (bench lines) + the fp8 / config-4 GPU tests
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_config4.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/cfg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/cfg_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 5 4; do
  timeout -k 10 400 python bench.py --config $c --steps 20 > $O/bench_c$c.log 2>&1 || exit 1
  echo "config $c: $(tail -1 $O/bench_c$c.log | cut -c1-400)"
done
