# Probe timelines of the replayed config-2 step (tools/step_timeline.py) under capture-order A/B
set -o pipefail
o=gpurun_out/timeline.log
: > $o
timeout -k 10 150 python -u tools/step_timeline.py >> $o 2>&1 || exit 1
EWVIT_MWT_FIRST=1 timeout -k 10 150 python -u tools/step_timeline.py >> $o 2>&1 || exit 1
EWVIT_BRANCH_STREAMS=0 timeout -k 10 150 python -u tools/step_timeline.py >> $o 2>&1 || exit 1
