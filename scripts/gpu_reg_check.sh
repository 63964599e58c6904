# after a change to the store paths: GPU tests (FILES, default all), then the registered leg's per-batch times
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-reg_check}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${FILES:-tests} > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 scripts/reg_trace.py registered > "$O/reg.json" 2>"$O/reg.err" || exit 1
python3 -c "import json;d=json.loads(open('$O/reg.json').read().strip().splitlines()[-1]);r=d['registered'];s=d['status_at_time_W'];print('registered dev', round(r['device_ms_per_batch'],4), 'count', round(r['count_ms_per_batch'],4), 'wall', round(r['compute_wall_ms_per_batch'],4), 'register', round(r['register_wall_ms_per_batch'],4), 'upload', round(r.get('upload_wall_ms_per_batch',0),4), '| status-at-time dev', round(s['device_ms_per_batch'],4), 'wall', round(s['compute_wall_ms_per_batch'],4))"
timeout -k 10 300 python3 scripts/reg_trace.py resident > "$O/res.json" 2>"$O/res.err" || exit 1
python3 -c "import json;d=json.loads(open('$O/res.json').read().strip().splitlines()[-1]);[print('resident', r['batches'], 'device', round(r['device_ms'],3), 'wall', round(r['compute_wall_ms'],3)) for r in d]"
