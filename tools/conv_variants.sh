#!/bin/bash
# conv kernel variants (EWVIT_CONV_BK / EWVIT_CONV_PF) on the step's conv shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
for V in "64 1" "64 2" "32 1" "32 2"; do
  set -- $V
  echo "== BK=$1 PF=$2" >> "$O/conv_variants.log"
  EWVIT_CONV_BK=$1 EWVIT_CONV_PF=$2 timeout -k 10 300 python "$R/tools/conv_bench.py" >> "$O/conv_variants.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
done
