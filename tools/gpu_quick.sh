#!/bin/bash
# Quick GPU iteration: selected GPU test files (TESTS), then the bench (skip with NOBENCH=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/quick_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$O/quick_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${NOBENCH:-0}" != 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$O/bench_quick.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 "$O/bench_quick.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
echo done
