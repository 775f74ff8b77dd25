# The fused DWT front end alone: timing (tools/dwt_bench.py) and its HBM traffic per launch
# from two separate rocprofv3 counter passes (FETCH_SIZE x2 on gfx950, WRITE_SIZE)
set -o pipefail
O=gpurun_out
timeout -k 10 120 python -u tools/dwt_bench.py > $O/dwt_xcd.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/dwtpmc_$C -o run -- python3 tools/dwt_bench.py --iters 5 --channels 9 > $O/dwtpmc_$C.log 2>&1 || exit 1
done
