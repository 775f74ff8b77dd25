# 32-wide column tiles for <= 32-column dgrads (EWVIT_CONV_BN32) on the stage-2/3 shapes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for V in 1 0; do
  echo "== BN32=$V"
  EWVIT_CONV_BN32=$V timeout -k 10 200 python "$R/tools/conv_bench.py" --only bb_s --iters 20 | grep glds1
done
