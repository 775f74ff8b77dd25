#!/bin/bash
# round 4: watchdog probe, the whole GPU suite, a bench line, the branch / token-path timings
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/fr_probe.py > $O/fr_probe.log 2>&1; echo "probe rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_dropin.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/head_tests.log 2>&1
rc=$?; echo "head tests rc=$rc"; tail -4 $O/head_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/branch_time.py --reps 20 --probe-us 500 --tables 40 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; tail -2 $O/branch_time.log; exit $rc
