cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_graph.py > $O/ts2j.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_s2j.log 2>&1 || exit 4
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_s2j.log 2>&1 || exit 5
