#!/bin/bash
# local helper (runs HERE, not on the GPU box): gpurun with retries while no box / slot is free
# usage: tools/gr.sh TIMEOUT_S OUTFILE -- command...
T=$1; OUT=$2; shift 3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT"; then sleep 60; continue; fi
  break
done
grep -v "every call sends" "$OUT" | tail -25
