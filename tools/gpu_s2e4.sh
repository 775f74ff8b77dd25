cd $GRAFT_REPO_ROOT
ENVS="EWVIT_SE_DX_FOLD=1 EWVIT_SE_DX_FOLD=0" timeout -k 10 700 bash tools/ab_env.sh 2 3 > gpurun_out/abs2e.log 2>&1 || exit 5
