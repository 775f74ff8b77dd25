# fp8 MXFP8 tests, config-5 bench, then the window non-temporal A/B on config 2
cd $GRAFT_REPO_ROOT
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_vit.py tests/test_gpu_head.py > gpurun_out/fp8_fused.log 2>&1
ok $? || exit 3
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_c5_mx.log 2>&1 || exit 4
ENVS="EWVIT_WIN_NT=0 EWVIT_WIN_NT=1" timeout -k 10 600 bash tools/ab_env.sh 2 2 > gpurun_out/ab_win_nt.log 2>&1 || exit 5
