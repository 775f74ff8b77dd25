#!/bin/bash
# hfsep forward with the next band's loads in flight during the MFMAs: tests, isolated timing
# against the previous build (ablib/libewvit_base.so), bench A/B interleaved
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_hfsep.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/hsab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/hsab_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in new base; do
  if [ $lib = base ]; then export EWVIT_LIB=$PWD/ablib/libewvit_base.so; else unset EWVIT_LIB; fi
  timeout -k 10 200 python tools/hfsep_bench.py > $O/hsab_iso_$lib.log 2>&1 || exit 1
  echo "iso $lib:"; grep -v amdgpu.ids $O/hsab_iso_$lib.log | tail -8
done
for r in 1 2; do for lib in new base; do
  if [ $lib = base ]; then export EWVIT_LIB=$PWD/ablib/libewvit_base.so; else unset EWVIT_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/hsab_b_$lib.log 2>&1 || exit 1
  echo "bench $lib $(tail -1 $O/hsab_b_$lib.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
