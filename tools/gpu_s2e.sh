# BN + SE dx pass folded into the depthwise backward (SeDxLink): parity tests, then the A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_reduce_defer.py tests/test_gpu_se.py tests/test_gpu_bn_link.py tests/test_abi.py > $O/ts2e.log 2>&1 || exit 3
ENVS="EWVIT_SE_DX_FOLD=1 EWVIT_SE_DX_FOLD=0" timeout -k 10 700 bash tools/ab_env.sh 2 3 > $O/abs2e.log 2>&1 || exit 5
