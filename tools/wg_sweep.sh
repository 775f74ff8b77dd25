# bench A/B sweep: the weight-gradient side stream (EWVIT_WGRAD_STREAM) x backward MWT cap
set -e
cd "$GRAFT_REPO_ROOT"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/wgs_$tag.log 2>&1
  echo "$tag: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/wgs_$tag.log').read().strip().splitlines()[-1]);print(d['value'])")"
}
for r in 1 2; do
  run base$r EWVIT_WGRAD_STREAM=0
  run wg_all$r EWVIT_WGRAD_STREAM=1 EWVIT_WGRAD_MIN_FLOPS=0
  run wg_all_bwd128_$r EWVIT_WGRAD_STREAM=1 EWVIT_WGRAD_MIN_FLOPS=0 EWVIT_MWT_GRID_CAP_BWD=128
  run wg_1e9_$r EWVIT_WGRAD_STREAM=1 EWVIT_WGRAD_MIN_FLOPS=1e9
done
