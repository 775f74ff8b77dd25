# same-box A/B of environment switches on config 2 (ENVS set by the caller), 2 interleaved rounds
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash tools/ab_env.sh 2 2 > gpurun_out/ab_knobs.log 2>&1 || exit 5
