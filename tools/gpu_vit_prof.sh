#!/bin/bash
# ViT tests, the ViT encoder micro-benchmark, plain and under rocprofv3 kernel stats
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/vit_tests.log 2>&1
rc=$?; echo "vit rc=$rc"; tail -2 $O/vit_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/vit_bench.py > $O/vit_bench.log 2>&1
rc=$?; echo "vb rc=$rc"; tail -1 $O/vit_bench.log; [ $rc -eq 0 ] || exit $rc
rm -rf $O/vitprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/vitprof -o vit -- python tools/vit_bench.py > $O/vit_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
