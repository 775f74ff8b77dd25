#!/bin/bash
# round-4 contract checks: watchdog probe, capture modes, drop-in tests, headline oracle
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/fr_probe.py > $O/fr_probe.log 2>&1; echo "probe rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s \
  tests/test_gpu_dp_graph.py tests/test_gpu_dropin.py tests/test_gpu_graph.py tests/test_gpu_bn_link.py \
  tests/test_gpu_headline_oracle.py > $O/contract.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 $O/contract.log; exit $rc
