# WaitingOn levelling check: GPU parity tests for a12/a13, a config-5 bench line, then the
# config-5 full-size parity test (FULL=0 skips it).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-wo}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "not full_size" tests/test_gpu_waiting_on.py > "$O/pytest_wo.log" 2>&1 && \
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > "$O/bench_c5.json" 2> "$O/bench_c5.err"
rc=$?; echo "rc=$rc"; tail -5 "$O/pytest_wo.log"; cat "$O/bench_c5.json"
[ $rc -ne 0 ] && exit $rc
[ "${FULL:-1}" = 0 ] && exit 0
timeout -k 10 600 python -u -m pytest -x -v --timeout 580 --timeout-method thread -m gpu -k "full_size" tests/test_gpu_waiting_on.py > "$O/pytest_wo_full.log" 2>&1
rc=$?; tail -3 "$O/pytest_wo_full.log"; exit $rc
