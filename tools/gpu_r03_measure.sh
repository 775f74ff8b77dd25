#!/bin/bash
# Round-3 measurement session: bench line, rocprofv3 kernel stats of the bench, which branch
# bounds the step (tools/branch_time.py with per-entry tables), and a kernel trace of the SFE
# (backbone + ViT head) piece alone.  Each GPU step under its own time limit, chained with &&.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$O/bench.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof.log" 2>&1)
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BRANCH:-0}" != 1 ]; then
  timeout -k 10 300 python tools/branch_time.py --reps 20 --tables 25 > "$O/branch_time.log" 2>&1
  rc=$?; echo "branch_time rc=$rc"; head -1 "$O/branch_time.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_PIECE:-0}" != 1 ]; then
  PIECE=${PIECE:-sfe} bash tools/gpu_piece_trace.sh
  rc=$?; echo "piece trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo done
