# the round-end run: GPU suite, configs 2/4/5, rocprofv3 kernel stats of config 2
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_final.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py > $O/bench_c2_final.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --config 4 --no-cpu-baseline > $O/bench_c4_final.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --config 5 --no-cpu-baseline > $O/bench_c5_final.log 2>&1 || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_final -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu-baseline > $O/prof_final.log 2>&1 || exit 7
rm -f $O/prof_final/run_kernel_trace.csv
