#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/head_tests.log 2>&1
rc=$?; echo "head tests rc=$rc"; grep -E "us per replay|passed|failed|Error" $O/head_tests.log | tail -5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run -- python -m pytest tests/test_gpu_head.py -q -k launch_time -p no:cacheprovider > $O/prof_head.log 2>&1
echo "prof rc=$?"; exit $rc
