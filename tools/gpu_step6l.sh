cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_se.py tests/test_gpu_bn_link.py > $O/t6l.log 2>&1 || exit 3
for r in 1 2; do
  for v in 0 1; do
    EWVIT_WIN_NT=$v timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --steps 20 > $O/ab6l_$v.log 2>&1 || exit 4
    echo "round=$r c4 win_nt=$v $(tail -1 $O/ab6l_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6l.log
  done
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6l_c2.log 2>&1 || exit 5
  echo "round=$r c2 se_fix $(tail -1 $O/ab6l_c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6l.log
done
