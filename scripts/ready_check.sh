# Readiness check: its GPU tests, the bench --registered --ready leg and a kernel trace of the
# readiness schedule (scripts/ready_run.py), the trace reduced to its stats and busy/idle split.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TAG=${TAG:-ready}; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ready.py tests/test_waiting_on_init.py tests/test_registered_schedule.py > "$O/pytest.log" 2>&1 && \
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --registered --ready > "$O/bench_registered.json" 2> "$O/bench_registered.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/tr" -o run --output-format csv -- python3 "$R/scripts/ready_run.py" > "$O/ready.log" 2>&1
rc=$?
[ -f "$O/tr/run_kernel_trace.csv" ] && python3 "$R/scripts/trace_gaps.py" "$O/tr/run_kernel_trace.csv" && rm -f "$O/tr/run_kernel_trace.csv"
tail -2 "$O/pytest.log"; exit $rc
