cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_win.py > $O/t6m.log 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --steps 20 > $O/ab6m_c4.log 2>&1 || exit 4
  echo "round=$r c4 $(tail -1 $O/ab6m_c4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6m.log
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6m_c2.log 2>&1 || exit 5
  echo "round=$r c2 $(tail -1 $O/ab6m_c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6m.log
  EWVIT_WIN_NT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6m_c2nt0.log 2>&1 || exit 5
  echo "round=$r c2 nt=0 $(tail -1 $O/ab6m_c2nt0.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6m.log
done
