# depthwise row kernel: columns loaded ahead DW_PD = 2 (default) vs 1 / 3 (A/B libraries); parity tests first
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bn_link.py tests/test_gpu_reduce_defer.py tests/test_gpu_modules.py > $O/ts2c.log 2>&1 || exit 3
ENVS="NONE=0 EWVIT_LIB=$GRAFT_REPO_ROOT/ab_lib/libewvit_pd1.so EWVIT_LIB=$GRAFT_REPO_ROOT/ab_lib/libewvit_pd3.so" timeout -k 10 900 bash tools/ab_env.sh 2 3 > $O/abs2c.log 2>&1 || exit 5
