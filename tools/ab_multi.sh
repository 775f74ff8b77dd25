# A/B of env sets (two interleaved rounds): bash tools/ab_multi.sh "A=1 B=2" "A=0 B=3" ...
O=gpurun_out; mkdir -p $O
for r in 1 2 3; do i=0; for v in "$@"; do i=$((i+1))
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $O/abm_$i.log 2>&1 || exit 1
  echo "[$v] $(tail -1 $O/abm_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done; done
