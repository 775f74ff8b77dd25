#!/bin/bash
# SQ counters of the windowed conv kernels (tools/win_bench.py --profile): one rocprofv3
# pass per counter set, --kernel-trace only (no sys/runtime trace with --pmc).
# Usage: tools/win_pmc.sh PHASE SHAPE VARIANTS "SET1" "SET2" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
PH=$1; SH=$2; VA=$3; shift 3
cd /tmp && export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/wpmc_${PH}_$i" -o run -- \
      python3 "$R/tools/win_bench.py" --only $SH --profile $PH --variants $VA > "$O/wpmc_${PH}_$i.log" 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
