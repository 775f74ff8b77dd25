#!/bin/bash
# round 4: branch timings, a bench line, and a rocprofv3 kernel trace of a short bench run
set -o pipefail
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/branch_time.py --reps 20 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; tail -1 $O/branch_time.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
rm -rf $O/prof_m
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_m -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_m.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
