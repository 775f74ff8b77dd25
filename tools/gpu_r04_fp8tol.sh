#!/bin/bash
# the fp8 DAMA-vs-oracle test's measured errors (EWVIT_PARITY_LOG) under three builds
set -o pipefail
O=gpurun_out; mkdir -p $O
for lib in pregate cur new; do
  case $lib in pregate) export EWVIT_LIB=$PWD/ablib/libewvit_pregate.so;; new) export EWVIT_LIB=$PWD/ablib/libewvit_new.so;; cur) unset EWVIT_LIB;; esac
  rm -f $O/fp8tol_$lib.jsonl
  EWVIT_PARITY_LOG=$PWD/$O/fp8tol_$lib.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -q --timeout 250 --timeout-method thread -p no:cacheprovider -k "oracle or chunks" > $O/fp8tol_$lib.log 2>&1
  echo "$lib rc=$? $(tail -1 $O/fp8tol_$lib.log)"
  grep -h "fused\|space\|freq" $O/fp8tol_$lib.jsonl | cut -c1-200
done
true
