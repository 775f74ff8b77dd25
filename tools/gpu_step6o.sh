# ewvit_bn_se_bwd (BN backward sums in the SE squeeze pass): parity tests, then the step A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_se.py tests/test_gpu_bn_link.py > $O/t6o.log 2>&1 || exit 3
ENVS="EWVIT_BN_SE_FUSED=1 EWVIT_BN_SE_FUSED=0" timeout -k 10 600 bash tools/ab_env.sh 2 3 > $O/ab6o.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p6o -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --no-cpu-baseline > $O/p6o.log 2>&1 || exit 7
