# A/B of the per-DMA window non-temporal mask (convwin.hip g_win_nt): 7 all, 1 fwd/dgrad only,
# 5 fwd/dgrad + wgrad x, 3 fwd/dgrad + wgrad dy, 0 none — config 2, three interleaved rounds
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_win.py > $O/t6n.log 2>&1 || exit 3
ENVS="EWVIT_WIN_NT=7 EWVIT_WIN_NT=1 EWVIT_WIN_NT=5 EWVIT_WIN_NT=3 EWVIT_WIN_NT=0" timeout -k 10 1000 bash tools/ab_env.sh 2 3 > $O/ab6n.log 2>&1 || exit 5
