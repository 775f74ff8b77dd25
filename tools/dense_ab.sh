# dense-K conv forward A/B (EWVIT_CONV_DENSE_W8MAX / EWVIT_CONV_DENSE_NS) on the stage-2/3 shapes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for V in "2048 2" "8192 2" "2048 3" "8192 3"; do
  set -- $V
  echo "== W8MAX=$1 NS=$2"
  EWVIT_CONV_DENSE_W8MAX=$1 EWVIT_CONV_DENSE_NS=$2 timeout -k 10 200 python "$R/tools/conv_bench.py" --only bb_s --iters 20
done
