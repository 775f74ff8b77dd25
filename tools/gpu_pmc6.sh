cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc6_c2.log 2>&1 || exit 3
BENCH_ARGS="--config 5" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc6_c5.log 2>&1 || exit 4
BENCH_ARGS="--config 4" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc6_c4.log 2>&1 || exit 5
