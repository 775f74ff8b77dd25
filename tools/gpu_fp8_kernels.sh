set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fp8.py -k "gemm" > gpurun_out/fp8_kernels.log 2>&1
