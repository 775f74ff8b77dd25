# usage: VAR=name bash ab.sh v1 v2 ...  (two rounds, interleaved)
O=gpurun_out; mkdir -p $O
for r in 1 2; do for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/ab_$v.log 2>&1 || exit 1
  echo "$VAR=$v $(tail -1 $O/ab_$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done; done
