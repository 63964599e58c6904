# registered-status path after a change: its GPU tests, then the registered leg's per-batch times
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-reg_check}"; mkdir -p "$O"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_registered_schedule.py tests/test_gpu_status_events.py tests/test_redundant_before.py tests/test_ready.py tests/test_waiting_on_init.py tests/test_gpu_resident.py > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 "$O/pytest.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 scripts/reg_trace.py registered > "$O/reg.json" 2>"$O/reg.err" || exit 1
python3 -c "import json;d=json.loads(open('$O/reg.json').read().strip().splitlines()[-1]);r=d['registered'];s=d['status_at_time_W'];print('registered dev', round(r['device_ms_per_batch'],4), 'count', round(r['count_ms_per_batch'],4), 'wall', round(r['compute_wall_ms_per_batch'],4), '| status-at-time dev', round(s['device_ms_per_batch'],4))"
TAG=r04_rk3 ENV_A="ACCORD_RK_BLOCKS=16384" ENV_B="ACCORD_RK_BLOCKS=32768" BENCH_ARGS="--config 3" bash scripts/gpu_env_ab.sh
