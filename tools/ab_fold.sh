set -o pipefail
for cfg in 2 4; do
for rep in 1 2; do
for v in "1 1" "1 0" "0 0"; do
  set -- $v
  r=$(EWVIT_FOLD_FUSION_BN=$1 EWVIT_BN_BWD_EPI=$2 timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "cfg $cfg fold $1 epi $2 rep $rep: $r"
done; done; done
