# Run a subset of GPU tests: FILES="tests/x.py ..." TAG=... bash scripts/gpu_tests.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-t}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${FILES:-tests} > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$O/pytest_gpu.log"; exit $rc
