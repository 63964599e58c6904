# Range-path parity (ranges + resident ranges) then the config-3 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-c3t}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ranges.py tests/test_gpu_accept.py ${EXTRA:-} > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
TAG=$TAG/p bash scripts/gpu_c3prof.sh
