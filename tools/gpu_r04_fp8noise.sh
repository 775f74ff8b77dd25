#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
for lib in pregate cur; do
  case $lib in pregate) export EWVIT_LIB=$PWD/ablib/libewvit_pregate.so;; cur) unset EWVIT_LIB;; esac
  echo "== $lib"
  timeout -k 10 300 python tools/fp8_noise.py > $O/fp8noise_$lib.log 2>&1 || { tail -5 $O/fp8noise_$lib.log; exit 1; }
  grep '^{' $O/fp8noise_$lib.log
done
