cd $GRAFT_REPO_ROOT
O=gpurun_out
for r in 1 2; do
  for cap in 80 96 112 128; do
    EWVIT_MWT_GRID_CAP=$cap timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/cap_$cap.log 2>&1 || exit 4
    echo "round=$r cap=$cap $(tail -1 $O/cap_$cap.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/cap_sweep6.log
  done
done
