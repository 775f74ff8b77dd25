# frame resize kernel: band height A/B (EWVIT_FRAMES_RB: the tallest band tried) and LDS budget
set -e
for r in 1 2; do for V in "8 64" "4 64" "2 64" "16 96"; do
  set -- $V
  echo "== RB $1 LDS $2 KB: $(EWVIT_FRAMES_RB=$1 EWVIT_FRAMES_LDS=$2 timeout -k 10 120 python tools/frames_bench.py --cpu-seconds 0.1 2>/dev/null | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["plan"], r["avg_us"], r["achieved_GBps"])')"
done; done
