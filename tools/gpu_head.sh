#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/fr_probe.py > $O/fr_probe.log 2>&1; echo "probe rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/head_tests.log 2>&1
rc=$?; echo "head tests rc=$rc"; tail -4 $O/head_tests.log; exit $rc
