# early optimizer step (TrainStep early_params): tests, then the A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_optim.py tests/test_gpu_reduce_defer.py > $O/ts2i.log 2>&1 || exit 3
ENVS="EWVIT_EARLY_STEP=1 EWVIT_EARLY_STEP=0" timeout -k 10 700 bash tools/ab_env.sh 2 3 > $O/abs2i.log 2>&1 || exit 5
