#!/bin/bash
# round 4 evidence: the whole GPU suite, smoke, bench line (with cpu_baseline), branch timings,
# rocprofv3 kernel stats of a bench run
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/branch_time.py --reps 20 --tables 30 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; head -2 $O/branch_time.log | tail -1; [ $rc -eq 0 ] || exit $rc
rm -rf $O/prof_r04c
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04c -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_r04c.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
