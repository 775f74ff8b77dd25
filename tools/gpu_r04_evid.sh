#!/bin/bash
# round 4 evidence: conv tests (weight packing), bench line, rocprofv3 kernel stats of a bench run
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_vit.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/conv_tests.log 2>&1
rc=$?; echo "conv rc=$rc"; tail -1 $O/conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_quick.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
rm -rf $O/prof_r04b
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04b -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_r04b.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $O/prof_r04b.log | cut -c1-200; exit $rc
