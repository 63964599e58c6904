set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04_eal"; mkdir -p "$O"
timeout -k 10 300 python3 -u scripts/dbg_eal.py > "$O/dbg.txt" 2>&1; echo "dbg rc=$?"; grep -m 3 "MISMATCH\|no mismatch" "$O/dbg.txt"; grep "wo-init-dbg" "$O/dbg.txt" | grep "dep 2104"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_waiting_on_init.py tests/test_gpu_resident.py tests/test_registered_schedule.py tests/test_redundant_before.py tests/test_gpu_status_events.py > "$O/pytest.log" 2>&1; echo "pytest rc=$?"; tail -3 "$O/pytest.log"
for v in 0 1; do
  ACCORD_RB_UNION=$v timeout -k 10 300 python3 scripts/reg_trace.py registered > "$O/reg_$v.json" 2>"$O/reg_$v.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/reg_$v.json').read().strip().splitlines()[-1]);r=d['registered'];print('rb_union=$v dev', round(r['device_ms_per_batch'],4), 'wall', round(r['compute_wall_ms_per_batch'],4), 'reg', round(r['register_wall_ms_per_batch'],4), 'rb', round(r['rb_wall_ms_per_batch'],4))"
done
