# Round 5, call b: the whole GPU suite (branch-free ts_cmp, executeAtLeast merge fix, removal spill pass)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${TAG:-r05_b}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ready.py tests > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
