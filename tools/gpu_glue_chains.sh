#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python tools/glue_chains.py > $O/glue_chains.log 2>&1; rc=$?; echo "rc=$rc"; tail -150 $O/glue_chains.log; exit $rc
