#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python tools/glue_chains.py 5 > $O/glue_chains_c5.log 2>&1; rc=$?; echo "rc=$rc"; exit $rc
