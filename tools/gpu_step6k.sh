cd $GRAFT_REPO_ROOT
O=gpurun_out
ROUNDS="1 2 3" timeout -k 10 1000 bash tools/lib_ab.sh > $O/ab_bn_pf.log 2>&1 || exit 6
