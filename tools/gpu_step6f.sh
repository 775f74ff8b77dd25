cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_conv_ksplit.py tests/test_gpu_bn_link.py tests/test_gpu_conv.py tests/test_gpu_wgrad_1x1.py > $O/t6f.log 2>&1 || exit 3
for r in 1 2 3; do
  for v in 0 1; do
    EWVIT_CONV_KSPLIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6f_$v.log 2>&1 || exit 4
    echo "round=$r ksplit=$v $(tail -1 $O/ab6f_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6f.log
  done
done
