# rocprofv3 kernel trace of one branch piece replayed from its own graph (tools/piece_trace.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=${PIECE:-sfe}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace -o run -- python3 tools/piece_trace.py --piece $P --reps 4 > gpurun_out/ptrace_$P.log 2>&1
f=$(find gpurun_out/ptrace -name '*kernel_trace.csv' | head -1)
M=stem_conv; [ "$P" = mwt ] && M=dwt_hf_fused
python3 tools/trace_step.py "$f" --marker $M --by-grid --nth 2 > gpurun_out/piece_${P}_by_grid.txt
python3 tools/trace_step.py "$f" --marker $M --all --nth 2 > gpurun_out/piece_${P}_all.txt
rm -rf gpurun_out/ptrace
