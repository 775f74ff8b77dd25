# Same-box sweep of the MWT workgroup cap: CAPS="128 160 192" bash tools/ab_cap.sh CONFIG REPS
set -o pipefail
cfg=${1:-2}; reps=${2:-2}
for rep in $(seq $reps); do
  for c in ${CAPS:-128 160 192}; do
    r=$(EWVIT_MWT_GRID_CAP=$c timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "cfg $cfg cap $c rep $rep: $r"
  done
done
