# the reworked MX GEMM + head MXFP8 test, config-5 bench, window NT A/B (3 reps)
cd $GRAFT_REPO_ROOT
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_head.py -k "gemm or mxfp8 or yardstick or precision or config5" > gpurun_out/fp8_b.log 2>&1
ok $? || exit 3
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_c5_mx2.log 2>&1 || exit 4
ENVS="EWVIT_WIN_NT=0 EWVIT_WIN_NT=1" timeout -k 10 900 bash tools/ab_env.sh 2 3 > gpurun_out/ab_win_nt2.log 2>&1 || exit 5
