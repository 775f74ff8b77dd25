# depthwise row kernels with 16 channel quads per block row (DW_Q16=1 A/B library) vs 8 (default);
# MWT cap 128 vs 96 on the default library.  Parity of the A/B library first.
cd $GRAFT_REPO_ROOT
O=gpurun_out
EWVIT_LIB=$GRAFT_REPO_ROOT/ab_lib/libewvit_q16.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bn_link.py tests/test_gpu_reduce_defer.py > $O/ts2d.log 2>&1 || exit 3
ENVS="NONE=0 EWVIT_LIB=$GRAFT_REPO_ROOT/ab_lib/libewvit_q16.so EWVIT_MWT_GRID_CAP=128" timeout -k 10 900 bash tools/ab_env.sh 2 3 > $O/abs2d.log 2>&1 || exit 5
