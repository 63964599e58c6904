# WaitingOn levelling check: GPU parity tests for a12/a13 and a config-5 bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-wo}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_waiting_on.py > "$O/pytest_wo.log" 2>&1 && \
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/bench_c5.json" 2> "$O/bench_c5.err"
rc=$?; echo "rc=$rc"; tail -5 "$O/pytest_wo.log"; cat "$O/bench_c5.json"; exit $rc
