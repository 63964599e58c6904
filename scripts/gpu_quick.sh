# Quick GPU iteration: all gpu tests, config-2 bench line, config-2 kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"
cd "$R"
TAG=${TAG:-quick}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
timeout -k 10 900 python -m pytest tests -x -q -m gpu > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS} > "$O/prof_trace.log" 2>&1
rc=$?
echo "rc=$rc"
tail -3 "$O/pytest_gpu.log"
exit $rc
