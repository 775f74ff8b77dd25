#!/bin/bash
# SQ counters of the conv kernels on one conv_bench shape (eager launches), one pass.
# Usage: SHAPE=mwt_multiscale bash tools/gpu_conv_pmc.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/conv_pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    -d "$O" -o pmc --output-format csv -- python3 "$R/tools/conv_bench.py" --only "${SHAPE:-mwt_multiscale}" \
    --variants 9 --rounds 1 --iters 3 --eager > "$O/log.txt" 2>&1
echo "pmc rc=$?"
