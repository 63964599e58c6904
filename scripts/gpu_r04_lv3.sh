set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_lv3"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; grep -m 3 "MISMATCH\|no mismatch" "$O/dbg.txt"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest_wo.log" 2>&1; rc=$?; echo "pytest wo rc=$rc"; tail -3 "$O/pytest_wo.log"; [ $rc -eq 0 ] || exit 1
ACCORD_LV_STATS=1 timeout -k 10 200 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu > "$O/c5.json" 2>"$O/c5.err" || { tail -5 "$O/c5.err"; exit 1; }
grep "lv stats" "$O/c5.err" | tail -1
python3 -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);s=d['stage_ms'];print('c5', round(d['ms_per_step'],3), 'wo_level', round(s['wo_level'],3))"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident.py tests/test_registered_schedule.py tests/test_ready.py > "$O/pytest.log" 2>&1; echo "pytest rc=$?"; tail -3 "$O/pytest.log"
