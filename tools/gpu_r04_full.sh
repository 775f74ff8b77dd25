#!/bin/bash
# round 4: the headline oracle test (prints every metric), then the whole GPU suite
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline_oracle.py -x -v -s --timeout 350 --timeout-method thread -p no:cacheprovider > $O/headline.log 2>&1
rc=$?; echo "headline rc=$rc"; tail -3 $O/headline.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_headline_oracle.py::test_headline_chunk_train_step_vs_oracle > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; exit $rc
