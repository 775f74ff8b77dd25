# deferred weight-gradient reductions: parity tests, then the step A/B (config 2, 3 rounds)
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_reduce_defer.py tests/test_gpu_wgrad_1x1.py tests/test_gpu_graph.py tests/test_gpu_bn_link.py > $O/ts2a.log 2>&1 || exit 3
ENVS="EWVIT_DEFER_REDUCE=1 EWVIT_DEFER_REDUCE=0" timeout -k 10 700 bash tools/ab_env.sh 2 3 > $O/abs2a.log 2>&1 || exit 5
