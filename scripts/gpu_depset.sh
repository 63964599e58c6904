# GPU check of the deps-set operations (union / slice / invert) through the C ABI.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/depset"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_depset.py > "$O/pytest.log" 2>&1
rc=$?
tail -30 "$O/pytest.log"
exit $rc
