# per-branch split of an eager step (rocprofv3 kernel trace; tools/branch_split.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bsplit -o run -- python3 bench.py --eager --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bsplit.log 2>&1
python3 tools/branch_split.py gpurun_out/bsplit/run_kernel_trace.csv > gpurun_out/branch_split.txt
rm -rf gpurun_out/bsplit
