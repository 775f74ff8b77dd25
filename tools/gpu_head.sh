#!/bin/bash
# fused-head replay time at 64 frames (graph), the head tests
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -m pytest "tests/test_gpu_head.py::test_head_launch_time" -x -q -s -p no:cacheprovider > $O/head_time.log 2>&1
rc=$?; echo "head rc=$rc"; grep "per replay" $O/head_time.log; exit $rc
