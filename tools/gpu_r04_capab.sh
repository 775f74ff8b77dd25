#!/bin/bash
# A/B: deep-ring / 8-wave variants for capped-grid conv launches (EWVIT_AB_CAPSG, EWVIT_AB_CAPWNS):
# the capped-walk tests with both on, branch_time's MWT-capped piece, then interleaved bench rounds
set -o pipefail
O=gpurun_out; mkdir -p $O
EWVIT_AB_CAPSG=1 EWVIT_AB_CAPWNS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_cap.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/capab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/capab_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "0 0" "1 0" "0 4" "1 4"; do set -- $v
  EWVIT_AB_CAPSG=$1 EWVIT_AB_CAPWNS=$2 timeout -k 10 200 python tools/branch_time.py --reps 10 > $O/capab_bt_$1_$2.log 2>&1 || exit 1
  echo "bt sg=$1 wns=$2 $(grep "^{" $O/capab_bt_$1_$2.log)"
done
for r in 1 2; do for v in "0 0" "1 0" "0 4" "1 4"; do set -- $v
  EWVIT_AB_CAPSG=$1 EWVIT_AB_CAPWNS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/capab_$1_$2.log 2>&1 || exit 1
  echo "bench sg=$1 wns=$2 $(tail -1 $O/capab_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
