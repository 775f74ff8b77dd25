# 1x1 weight-gradient split rule after the deferred reductions: workgroup target / min K-tiles
cd $GRAFT_REPO_ROOT
ENVS="NONE=0 EWVIT_W1X1=128:8 EWVIT_W1X1=192:8 EWVIT_W1X1=384:8 EWVIT_W1X1=256:16" timeout -k 10 1000 bash tools/ab_env.sh 2 2 > gpurun_out/abs2k.log 2>&1 || exit 5
