#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/vit_tests.log 2>&1
rc=$?; echo "vit rc=$rc"; tail -1 $O/vit_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/pe_bench.py > $O/pe_bench.log 2>&1
rc=$?; echo "pe rc=$rc"; tail -1 $O/pe_bench.log; exit $rc
