cd $GRAFT_REPO_ROOT
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_head.py tests/test_gpu_fp8.py -k "mxfp8 or gemm" > gpurun_out/head_mx.log 2>&1
ok $? || exit 3
timeout -k 10 120 python -u tools/mx_gemm_bench.py > gpurun_out/mx_gemm_bench.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_c5_mx3.log 2>&1 || exit 5
