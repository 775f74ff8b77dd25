# One-stream, uncapped kernel trace of the config-2 step (rocprofv3 --kernel-trace) and its
# per-launch-configuration breakdown: python tools/trace_step.py ... --by-grid
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
EWVIT_BRANCH_STREAMS=0 EWVIT_MWT_GRID_CAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace1 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/trace1.log 2>&1
f=$(find gpurun_out/trace1 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_step.py "$f" --by-grid --largest > gpurun_out/step_by_grid.txt
python3 tools/trace_step.py "$f" --largest > gpurun_out/step_by_kernel.txt
rm -rf gpurun_out/trace1
