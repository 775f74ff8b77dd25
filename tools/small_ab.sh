# small-channel conv band height / LDS budget A/B (EWVIT_CONV_SMALL_TH / EWVIT_CONV_SMALL_LDS)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for V in "4 40" "2 40" "6 64" "8 64" "12 64"; do
  set -- $V
  echo "== TH=$1 LDS=$2"
  EWVIT_CONV_SMALL_TH=$1 EWVIT_CONV_SMALL_LDS=$2 timeout -k 10 200 python "$R/tools/conv_bench.py" --variants 9 --only s1_fused --iters 20 | grep glds
  EWVIT_CONV_SMALL_TH=$1 EWVIT_CONV_SMALL_LDS=$2 timeout -k 10 200 python "$R/tools/conv_bench.py" --variants 9 --only seperate --iters 20 | grep glds
done
