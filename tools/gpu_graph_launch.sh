# Host-launch vs device time of the replayed config-2 step under runtime / capture-order knobs
# (tools/graph_launch.py), then a kernel trace of the MWT-first capture for its timeline.
set -o pipefail
o=gpurun_out/graph_launch2.log
: > $o
timeout -k 10 150 python -u tools/graph_launch.py >> $o 2>&1 || exit 1
EWVIT_MWT_FIRST=1 timeout -k 10 150 python -u tools/graph_launch.py >> $o 2>&1 || exit 1
timeout -k 10 150 python -u tools/graph_launch.py >> $o 2>&1 || exit 1
EWVIT_MWT_FIRST=1 timeout -k 10 150 python -u tools/graph_launch.py >> $o 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
EWVIT_MWT_FIRST=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_mf -o run -- python3 tools/graph_launch.py --steps 4 > gpurun_out/prof_mf.log 2>&1
