# backward-only MWT cap at forward cap 128 (the MWT backward ends ~3.5 ms before the backbone's)
cd $GRAFT_REPO_ROOT
ENVS="NONE=0 EWVIT_MWT_BWD_CAP=96 EWVIT_MWT_BWD_CAP=80 EWVIT_MWT_BWD_CAP=64" timeout -k 10 900 bash tools/ab_env.sh 2 2 > gpurun_out/abs2m.log 2>&1 || exit 5
