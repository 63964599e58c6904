# Round 5, call o: event-exact readiness mode (ACCORD_READY_EVENTS) -- readiness GPU tests
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_o}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ready.py -k "event or propagate or kat" > "$O/pytest_ev.log" 2>&1 || { grep -E "FAIL|Error|assert" "$O/pytest_ev.log" | head -30; tail -40 "$O/pytest_ev.log"; exit 1; }
tail -3 "$O/pytest_ev.log"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ready.py tests/test_registered_schedule.py tests/test_gpu_status_events.py tests/test_waiting_on_init.py > "$O/pytest_gpu.log" 2>&1 || { grep -E "FAIL|Error|assert" "$O/pytest_gpu.log" | head -30; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
