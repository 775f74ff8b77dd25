cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/step_timeline.py > gpurun_out/timeline_s2l.log 2>&1 || exit 3
EWVIT_MWT_GRID_CAP=96 timeout -k 10 200 python -u tools/step_timeline.py >> gpurun_out/timeline_s2l.log 2>&1 || exit 4
