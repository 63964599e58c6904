# round-4: eal debug prints; levelling (split-role resolver) parity and config-5 A/B against the old walk
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_lv"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; grep -m 40 "eal-dbg\|MISMATCH" "$O/dbg.txt"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest_wo.log" 2>&1; rc=$?; echo "pytest wo rc=$rc"; tail -5 "$O/pytest_wo.log"; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  ACCORD_LV_OLD=$v timeout -k 10 200 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/c5_$v.json" 2>"$O/c5_$v.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('old=$v', round(d['ms_per_step'],3), 'wo_level', round(s['wo_level'],3), 'wo_preds', round(s['wo_preds'],3))"
done
