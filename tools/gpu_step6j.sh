cd $GRAFT_REPO_ROOT
O=gpurun_out
for r in 1 2; do
  for v in 96:0 96:80 96:88 96:112 128:88 128:96; do
    f=${v%%:*}; b=${v##*:}
    EWVIT_MWT_GRID_CAP=$f EWVIT_MWT_BWD_CAP=$b timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6j.json.log 2>&1 || exit 4
    echo "round=$r fwdcap=$f bwdcap=$b $(tail -1 $O/ab6j.json.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6j.log
  done
done
