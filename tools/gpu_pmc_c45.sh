# PMC refresh (FETCH_SIZE / WRITE_SIZE passes) for configs 5 and 4 on the current build
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--config 5" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc_c5.log 2>&1 || exit 3
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
BENCH_ARGS="--config 4" timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc_c4.log 2>&1 || exit 4
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
