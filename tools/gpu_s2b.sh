# MWT grid cap re-sweep after the deferred reductions (config 2, 2 rounds) + step timeline
cd $GRAFT_REPO_ROOT
O=gpurun_out
ENVS="EWVIT_MWT_GRID_CAP=96 EWVIT_MWT_GRID_CAP=112 EWVIT_MWT_GRID_CAP=128 EWVIT_MWT_GRID_CAP=80" timeout -k 10 700 bash tools/ab_env.sh 2 2 > $O/abs2b.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/step_timeline.py > $O/timeline_s2b.log 2>&1 || exit 6
