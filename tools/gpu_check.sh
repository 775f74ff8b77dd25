#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script
# (test *failures*, pytest rc 1, do not).  Outputs land in gpurun_out/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
STEPS=${STEPS:-all}

if [[ $STEPS == all || $STEPS == *tests* ]]; then
  rm -f "$O/parity.jsonl"
  EWVIT_PARITY_LOG="$O/parity.jsonl" timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > "$O/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  BL=${BENCH_LOG:-bench.log}
  timeout -k 10 600 python "$R/bench.py" ${BENCH_ARGS:-} > "$O/$BL" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 "$O/$BL" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo done
