#!/bin/bash
# conv wgrad reduce with up to 4x the split lanes (256K threads) (ablib/libewvit_new.so)
# against the in-tree build: SE / module / layer-by-layer tests, SFE piece and bench interleaved
set -o pipefail
O=gpurun_out; mkdir -p $O
EWVIT_LIB=$PWD/ablib/libewvit_new.so timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_layerwise.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/wrt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/wrt_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for lib in new base; do
  if [ $lib = new ]; then export EWVIT_LIB=$PWD/ablib/libewvit_new.so; else unset EWVIT_LIB; fi
  timeout -k 10 300 python tools/branch_time.py --reps 10 > $O/wrt_bt_$lib.log 2>&1 || exit 1
  echo "bt $lib $(grep '^{' $O/wrt_bt_$lib.log)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/wrt_b_$lib.log 2>&1 || exit 1
  echo "bench $lib $(tail -1 $O/wrt_b_$lib.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
