#!/bin/bash
# A/B of an env switch on the SFE piece: graph-replayed SFE fwd+bwd time (tools/branch_time.py's
# sfe_ms) for each setting of VAR in VALS, ROUNDS rounds interleaved.
set -u
O=gpurun_out; mkdir -p $O
for r in ${ROUNDS:-1 2}; do for v in ${VALS:-0 1}; do
  env $VAR=$v timeout -k 10 300 python tools/branch_time.py --reps 20 > $O/pab_${VAR}_$v.log 2>&1 || exit 1
  echo "$VAR=$v $(tail -1 $O/pab_${VAR}_$v.log)"
done; done
