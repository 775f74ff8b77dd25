#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_oracle.py -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/headline.log 2>&1
rc=$?; echo "headline rc=$rc"; tail -4 $O/headline.log; exit $rc
