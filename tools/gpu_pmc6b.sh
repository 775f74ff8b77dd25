cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc6b_c2.log 2>&1 || exit 3
rm -rf gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
