set -u
O=gpurun_out; mkdir -p $O
for sg in 0 8 9; do
  EWVIT_CONV_SG=$sg timeout -k 10 200 python tools/conv_bench.py --only bb_ --variants 1 --iters 20 $( [ $sg = 0 ] && echo --mm ) > $O/cb_sg$sg.log 2>&1 || exit 1
  echo "== SG=$sg"; grep -v amdgpu.ids $O/cb_sg$sg.log
done
