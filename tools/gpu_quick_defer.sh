cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reduce_defer.py tests/test_gpu_graph.py tests/test_gpu_dropin.py tests/test_gpu_headline_oracle.py > gpurun_out/ts3.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_s3.log 2>&1 || exit 4
