# Round 5, call p: event-exact readiness, one event per registration
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_p}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_ready.py -k "event or rb" > "$O/pytest_ev.log" 2>&1 || { grep -E "FAIL|Error|assert" "$O/pytest_ev.log" | head -30; tail -40 "$O/pytest_ev.log"; exit 1; }
tail -8 "$O/pytest_ev.log"
