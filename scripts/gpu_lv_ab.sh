# Levelling A/B: the config-5 level stage under each env setting (VARIANTS, ';'-separated), with the
# staged resolver's cycle stats (round 1; round 2 without them), after the WaitingOn GPU tests under the last setting.
#   TAG=... VARIANTS="ACCORD_LV_BCAST=0;ACCORD_LV_BCAST=1" bash scripts/gpu_lv_ab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-lv_ab}"; mkdir -p "$O"
IFS=';' read -ra VS <<< "${VARIANTS:-ACCORD_LV_BCAST=0;ACCORD_LV_BCAST=1}"
last="${VS[${#VS[@]}-1]}"
env $last timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for round in 1 2; do
  i=0
  for v in "${VS[@]}"; do
    env $v ACCORD_LV_STATS=$((2 - round)) timeout -k 10 200 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/v$i.$round.json" 2> "$O/v$i.$round.err" || { echo "$v failed"; tail -5 "$O/v$i.$round.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/v$i.$round.json').read().strip().splitlines()[-1]);print('$v', 'wo_level', round(d['stage_ms']['wo_level'],3))"
    grep lv_staged "$O/v$i.$round.err" | tail -1
    i=$((i+1))
  done
done
