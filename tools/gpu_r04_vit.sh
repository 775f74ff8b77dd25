#!/bin/bash
# round 4: fused ViT layer tests, the whole GPU suite (uncaptured output), bench, branch timings
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/vit_tests.log 2>&1
rc=$?; echo "vit rc=$rc"; tail -3 $O/vit_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/branch_time.py --reps 20 --tables 30 > $O/branch_time.log 2>&1
rc=$?; echo "branch rc=$rc"; head -1 $O/branch_time.log; exit $rc
