# MaxConflicts fold on one MI355X: its GPU tests, then the whole GPU suite, then a config-2 timing.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/mc"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_max_conflicts.py > "$O/pytest_mc.log" 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 200 python -u scripts/mc_timing.py > "$O/timing.log" 2>&1
rc=$?; tail -3 "$O/pytest_mc.log"; tail -2 "$O/pytest_gpu.log"; cat "$O/timing.log"; exit $rc
