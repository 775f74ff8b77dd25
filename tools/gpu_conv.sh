#!/bin/bash
# conv kernels: parity tests on both kernel families, then the A/B micro-benchmark.
# Test failures (rc 1) still run the bench; a crash/timeout ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_conv.py" -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$O/conv_tests.log" 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -3 "$O/conv_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u "$R/tools/conv_bench.py" ${CONV_BENCH_ARGS:-} > "$O/conv_bench.log" 2>&1
rc=$?; echo "conv bench rc=$rc"; cat "$O/conv_bench.log"; exit $rc
