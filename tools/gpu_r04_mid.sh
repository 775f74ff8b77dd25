#!/bin/bash
# round 4 mid-point: the whole GPU suite, a bench line and the branch / token-path timings
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/branch_time.py --reps 20 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; tail -1 $O/branch_time.log; exit $rc
