# readiness after a change: its GPU tests, then the --ready leg (scripts/reg_trace.py ready) timing
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-ready_check}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_waiting_on_init.py > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 scripts/reg_trace.py ready > "$O/ready.json" 2>"$O/ready.err" || exit 1
python3 -c "import json;d=json.loads(open('$O/ready.json').read().strip().splitlines()[-1]);print('ready ms/call', round(d['update_ms_per_call'],4), 'calls', d['update_calls'], 'apply ms total', round(d['apply_register_ms_total'],1))"
for v in 1 0 1 0; do
  ACCORD_READY_RESEND=$v timeout -k 10 300 python3 scripts/reg_trace.py ready > "$O/ready_$v.json" 2>"$O/ready_$v.err" || exit 1
  python3 -c "import json;d=json.loads(open('$O/ready_$v.json').read().strip().splitlines()[-1]);print('resend=$v ready ms/call', round(d['update_ms_per_call'],4))"
done
