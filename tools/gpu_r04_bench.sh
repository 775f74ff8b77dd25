#!/bin/bash
# round 4: a bench line and the branch / token-path timings
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/branch_time.py --reps 20 --probe-us 500 --tables 40 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; tail -2 $O/branch_time.log; exit $rc
