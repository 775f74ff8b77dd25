# A/B of the grouped seperate conv (EWVIT_HFSEP=1) against the block-diagonal dense conv (0):
# branch timing + bench, interleaved, same box
set -e
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in 0 1; do
    EWVIT_HFSEP=$v timeout -k 10 300 python tools/branch_time.py --reps 10 > gpurun_out/hsab_bt_${v}_${r}.log 2>&1
    echo "hfsep=$v round $r: $(tail -1 gpurun_out/hsab_bt_${v}_${r}.log)"
    EWVIT_HFSEP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/hsab_b_${v}_${r}.log 2>&1
    echo "hfsep=$v round $r: $(tail -1 gpurun_out/hsab_b_${v}_${r}.log | cut -c1-120)"
  done
done
