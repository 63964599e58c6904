# Round 5, call n: setAppliedAndPropagate on the device -- readiness / registered-schedule / status GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_n}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_registered_schedule.py tests/test_gpu_status_events.py tests/test_waiting_on_init.py > "$O/pytest_gpu.log" 2>&1 || { grep -E "FAIL|Error|assert" "$O/pytest_gpu.log" | head -30; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
