cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_conv_ksplit.py > $O/t6h.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/step_timeline.py --steps 7 > $O/timeline6h.log 2>&1 || exit 4
