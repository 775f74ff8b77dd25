# Round checkpoint on one GPU box: the GPU test suite, the config-2 bench (with the CPU baseline),
# config 4 and 5 bench lines, and a rocprofv3 kernel-stats pass of the config-2 bench.
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/rc_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/rc_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/rc_bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > $O/rc_bench_c5.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rc_prof -o run -- python3 bench.py --no-cpu-baseline > $O/rc_prof.log 2>&1
