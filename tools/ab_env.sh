# Same-box A/B of environment switches on the bench: ENVS="A=0 A=1" bash tools/ab_env.sh CONFIG REPS
# (each word of ENVS is one variant; a variant may join several assignments with commas)
set -o pipefail
cfg=${1:-2}; reps=${2:-2}
for rep in $(seq $reps); do
  for e in ${ENVS:-NONE=0}; do
    r=$(env ${e//,/ } timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "cfg $cfg $e rep $rep: $r"
  done
done
