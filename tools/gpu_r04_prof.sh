#!/bin/bash
# round 4: token-path timing with the fused head, and the rocprofv3 summary of a bench run
set -o pipefail
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/branch_time.py --reps 20 --tables 45 > $O/branch_time_r04.log 2>&1
rc=$?; echo "branch rc=$rc"; head -1 $O/branch_time_r04.log | tail -c 400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_r04 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_r04.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_r04.log | cut -c1-200; exit $rc
