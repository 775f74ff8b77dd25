# MWT caps above 128 (the MWT backward finishing earlier lets the backbone's last ms run alone)
cd $GRAFT_REPO_ROOT
ENVS="NONE=0 EWVIT_MWT_GRID_CAP=160 EWVIT_MWT_GRID_CAP=192 EWVIT_MWT_BWD_CAP=160 EWVIT_MWT_BWD_CAP=192" timeout -k 10 1000 bash tools/ab_env.sh 2 2 > gpurun_out/abs2n.log 2>&1 || exit 5
