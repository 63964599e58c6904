# Range-path GPU parity tests + config-3 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ranges.py tests/test_gpu_depset.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
TAG=$TAG bash scripts/gpu_c3prof.sh
