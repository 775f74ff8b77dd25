# full GPU suite on the current tree (from the fold test on) + config-2 bench
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_bn_link.py > $O/ts2f.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_s2f.log 2>&1 || exit 4
