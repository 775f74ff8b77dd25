#!/bin/bash
# PMC pass over the fused ViT encoder micro-benchmark (kernel trace + one counter set)
set -o pipefail
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/vitpmc
VIT_BENCH_MODES=1 timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum -d $O/vitpmc -o pmc -- python tools/vit_bench.py --iters 5 > $O/vit_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
