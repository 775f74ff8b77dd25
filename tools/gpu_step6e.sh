cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_bn_link.py tests/test_gpu_fp8.py tests/test_gpu_kernels.py > $O/t6e.log 2>&1 || exit 3
for r in 1 2 3; do
  for v in old nofuse new; do
    L=; F=1
    [ $v = old ] && L=$PWD/ab_lib/libewvit_old.so && F=0
    [ $v = nofuse ] && F=0
    EWVIT_LIB=$L EWVIT_DW_BWD_FUSED=$F timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab6e_$v.log 2>&1 || exit 4
    echo "round=$r lib=$v $(tail -1 $O/ab6e_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab6e.log
  done
done
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > $O/bench_c5_6e.log 2>&1 || exit 5
