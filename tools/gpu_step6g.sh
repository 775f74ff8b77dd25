cd $GRAFT_REPO_ROOT
O=gpurun_out
# EWVIT_CONV_KSPLIT: 0 off; 1 default (S <= 2, >= 8 K-tiles); 16*minkt + maxS
for r in 1 2; do
  for v in 0 1 66 132; do
    EWVIT_CONV_KSPLIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6g_$v.log 2>&1 || exit 4
    echo "round=$r ksplit=$v $(tail -1 $O/ab6g_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6g.log
  done
done
