#!/bin/bash
# HBM traffic per kernel: two separate rocprofv3 counter passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), each with --kernel-trace only.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
# a counter pass serialises ~1500 dispatches per step and prints nothing until it ends:
# report the growth of its output directory once a minute so the run is seen alive
( while sleep 60; do du -sk "$O"/pmc_* 2>/dev/null | tr '\n' ' ' >> "$O/pmc_progress.log"; echo >> "$O/pmc_progress.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/pmc_$C" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
F=$(ls "$O"/pmc_FETCH_SIZE/*counter_collection.csv | head -1)
W=$(ls "$O"/pmc_WRITE_SIZE/*counter_collection.csv | head -1)
CFG=$(echo "${BENCH_ARGS:-}" | sed -n 's/.*--config[ =]\([0-9]\).*/\1/p'); CFG=${CFG:-2}
python3 "$R/tools/pmc_summary.py" "$F" "$W" --steps 6 --config $CFG > "$O/pmc_summary_c$CFG.json" && echo pmc summary ok
