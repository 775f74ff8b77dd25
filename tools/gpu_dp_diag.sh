#!/bin/bash
# the GPU suite up to and including the data-parallel graph tests, uncaptured output
set -o pipefail
O=gpurun_out; mkdir -p $O
FILES=$(ls tests/test_*.py | sort | awk '{print} /test_gpu_dp_graph.py/ {exit}')
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dp_diag.log 2>&1
rc=$?; echo "dp rc=$rc"; tail -2 $O/dp_diag.log; exit $rc
