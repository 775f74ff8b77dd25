#!/bin/bash
# config 5 under rocprofv3 kernel trace: per-dispatch durations of the stage-6 BatchNorm/SE backward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/c5prof -o run -- python3 bench.py --config 5 --steps 10 --no-cpu-baseline > $O/c5prof.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $O/c5prof.log | cut -c1-200; exit $rc
