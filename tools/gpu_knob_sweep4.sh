# same-box A/B of environment switches on config 4 (ENVS set by the caller), 2 interleaved rounds
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash tools/ab_env.sh 4 2 > gpurun_out/ab_knobs4.log 2>&1 || exit 5
