#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/glue_sources.py > $O/glue.log 2>&1
rc=$?; echo "glue rc=$rc"; exit $rc
