# fused DWT -> HF upsample: threads / strip rows per workgroup A/B (EWVIT_DWTF_THREADS, EWVIT_DWTF_ROWS)
set -e
for r in 1 2; do for V in "256 16" "512 16" "256 8" "512 8" "512 32" "1024 32"; do
  set -- $V
  echo "== threads $1 rows $2: $(EWVIT_DWTF_THREADS=$1 EWVIT_DWTF_ROWS=$2 timeout -k 10 120 python tools/dwt_bench.py 2>/dev/null | tail -1)"
done; done
