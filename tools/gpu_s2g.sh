# full GPU suite + bench, then stream-priority A/B (backbone capture stream high / MWT stream high)
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/ts2f.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_s2f.log 2>&1 || exit 4
ENVS="NONE=0 EWVIT_MAIN_STREAM_PRIORITY=-1 EWVIT_MWT_STREAM_PRIORITY=-1" timeout -k 10 700 bash tools/ab_env.sh 2 2 > $O/abs2g.log 2>&1 || exit 5
