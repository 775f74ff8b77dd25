cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 200 python -u tools/step_timeline.py --steps 7 > $O/tl_96.log 2>&1 || exit 4
EWVIT_MWT_GRID_CAP=128 timeout -k 10 200 python -u tools/step_timeline.py --steps 7 > $O/tl_128.log 2>&1 || exit 4
EWVIT_MWT_GRID_CAP=64 timeout -k 10 200 python -u tools/step_timeline.py --steps 7 > $O/tl_64.log 2>&1 || exit 4
