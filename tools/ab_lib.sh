# Same-box A/B of bench.py over library builds / switches:
#   VARIANTS="cur head A B small0" bash tools/ab_lib.sh CONFIG REPS
# cur: the tree's libewvit.so; small0: it with 64-row glds tiles off; anything else: ab_lib/libewvit_<name>.so
set -o pipefail
cfg=${1:-2}; reps=${2:-2}
for rep in $(seq $reps); do
  for v in ${VARIANTS:-cur head small0}; do
    case $v in
      cur) envs="";;
      small0) envs="EWVIT_SMALL_TILES=0";;
      *) envs="EWVIT_LIB=$PWD/ab_lib/libewvit_$v.so";;
    esac
    r=$(env $envs timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "cfg $cfg $v rep $rep: $r"
  done
done
