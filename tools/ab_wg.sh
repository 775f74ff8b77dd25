# wgrad-stream A/B: off, then on at each minimum-FLOP threshold given
O=gpurun_out; mkdir -p $O
for v in off "$@"; do
  if [ $v = off ]; then E="EWVIT_WGRAD_STREAM=0"; else E="EWVIT_WGRAD_STREAM=1 EWVIT_WGRAD_MIN_FLOPS=$v"; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/abwg_$v.log 2>&1 || exit 1
  echo "$E $(tail -1 $O/abwg_$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
