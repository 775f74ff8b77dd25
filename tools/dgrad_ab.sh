# dgrad A/B on the stage-2/3 shapes: 256-row blocks (EWVIT_CONV_DG256), 8-wave threshold (EWVIT_CONV_W8MAX)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for V in "1024 2048" "0 2048" "0 8192" "1024 8192"; do
  set -- $V
  echo "== DG256=$1 W8MAX=$2"
  EWVIT_CONV_DG256=$1 EWVIT_CONV_W8MAX=$2 timeout -k 10 200 python "$R/tools/conv_bench.py" --only bb_s --iters 20 | grep glds1
done
