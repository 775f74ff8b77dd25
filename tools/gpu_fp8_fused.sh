set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_vit.py tests/test_gpu_head.py > gpurun_out/fp8_fused.log 2>&1
