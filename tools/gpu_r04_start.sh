#!/bin/bash
# round 4 (second session): dp-graph tests uncaptured, GPU suite, a bench line, the bench with one stream / uncapped grids
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_graph.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dp_diag.log 2>&1
rc=$?; echo "dp rc=$rc"; tail -2 $O/dp_diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
EWVIT_BRANCH_STREAMS=0 EWVIT_MWT_GRID_CAP=0 timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_1s.log 2>&1
rc=$?; echo "bench1s rc=$rc"; tail -1 $O/bench_1s.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/branch_time.py --reps 20 --tables 30 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; exit $rc
